"""Data-parallel gradient averaging / parameter broadcast over gloo, 2 ranks on CPU.

Exercises exactly the code the RCCL path runs (vgan.dist.GradSync over
vgan.flat.FlatParams); only the backend differs."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys

    from parity_util import PKG_ROOT
    sys.path.insert(0, PKG_ROOT)
    from vgan.dist import GradSync
    from vgan.flat import FlatParams

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different init on every rank
    net = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Tanh(), torch.nn.Linear(7, 3))
    flat = FlatParams(net)
    sync = GradSync()
    sync.broadcast_params(flat)
    x = torch.randn(11, 5) * (rank + 1)
    flat.zero_grad()
    net(x).pow(2).sum().backward()
    local = flat.grad.clone()
    sync.all_reduce_grad(flat)
    gathered = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(gathered, local)
    q.put((rank, flat.param.clone(), flat.grad.clone(), torch.stack(gathered).mean(0)))
    dist.destroy_process_group()


def test_gloo_two_ranks_average_and_broadcast():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, p0, g0, m0), (_, p1, g1, _) = res
    assert torch.equal(p0, p1)  # parameters broadcast from rank 0
    assert torch.allclose(g0, g1) and torch.allclose(g0, m0, atol=1e-6)  # averaged gradient
