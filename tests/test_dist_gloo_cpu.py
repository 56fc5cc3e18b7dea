"""Data-parallel gradient averaging / parameter broadcast over gloo, 2 ranks on CPU.

Exercises exactly the code the RCCL path runs (vgan.dist.GradSync over
vgan.flat.FlatParams); only the backend differs."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import pytest


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
    # plain data: a tensor travels as a file descriptor that dies with this process
    q.put((rank, flat.param.tolist(), flat.grad.tolist(), torch.stack(gathered).mean(0).tolist()))
    dist.destroy_process_group()


def _run(target, world=2):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_gloo_two_ranks_average_and_broadcast():
    (_, p0, g0, m0), (_, p1, g1, _) = _run(_worker)
    p0, g0, m0, p1, g1 = (torch.tensor(v) for v in (p0, g0, m0, p1, g1))
    assert torch.equal(p0, p1)  # parameters broadcast from rank 0
    assert torch.allclose(g0, g1) and torch.allclose(g0, m0, atol=1e-6)  # averaged gradient


def _trainer_worker(rank, world, port, q):
    """bench.py's order: per-rank CPU seed, then the models after the SAME
    torch.manual_seed(SEED) -- the rank must still reach the Trainer's RNG."""
    import sys

    from parity_util import PKG_ROOT
    sys.path.insert(0, PKG_ROOT)
    from vgan import dist as vdist
    from vgan.config import Configuration
    from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
    from vgan.trainer import Trainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    cfg = Configuration()
    cfg.DEVICE = "cpu"
    vdist.init("gloo", configuration=cfg)
    assert cfg.runtime["rank"] == rank and cfg.runtime["world_size"] == world
    cfg.runtime["rank"] = 0  # the process group, not a stale runtime entry, decides
    torch.manual_seed(cfg.SEED + rank)
    torch.manual_seed(cfg.SEED)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    tr = Trainer(G, D, None, og, od, None, cfg)
    means = tr.sync.all_reduce_scalars(torch.tensor([float(rank), 2.0 * rank]))
    q.put((rank, tr.rank, tr.rng.seed, means.tolist()))  # plain data: the worker exits before the parent reads
    dist.destroy_process_group()


def test_gloo_ranks_draw_different_streams():
    (_, r0, s0, m0), (_, r1, s1, m1) = _run(_trainer_worker)
    assert (r0, r1) == (0, 1)
    assert s0 != s1  # per-rank z / dropout / Gumbel / eps streams
    assert m0 == m1 == [0.5, 1.0]  # logged losses averaged


def test_sharded_loader_equal_steps_shared_shuffle():
    """Uneven batch count (11 batches, 2 ranks): every rank gets the same
    number of batches, ranks are disjoint, and the plan does not depend on the
    global CPU RNG (ranks seed it differently)."""
    import sys

    from parity_util import PKG_ROOT
    if PKG_ROOT not in sys.path:
        sys.path.insert(0, PKG_ROOT)
    from vgan.loader import GraphLoader

    indices = list(range(100, 141))  # 41 buildings -> 11 batches of 4 (drop_last=False)
    plans = []
    for rank in range(2):
        torch.manual_seed(777 + rank)
        ld = GraphLoader(None, indices, batch_size=4, rank=rank, world_size=2, seed=777)
        plans.append(ld.batches())
        assert len(ld) == len(plans[-1]) == 5
    flat0 = [i for b in plans[0] for i in b]
    flat1 = [i for b in plans[1] for i in b]
    assert not set(flat0) & set(flat1)
    assert len(flat0) + len(flat1) == 40  # the tail batch is cut, never split unevenly
    # next epoch reshuffles identically on both ranks
    a = GraphLoader(None, indices, batch_size=4, rank=0, world_size=2, seed=777)
    b = GraphLoader(None, indices, batch_size=4, rank=1, world_size=2, seed=777)
    torch.manual_seed(1)
    e1a = a.batches(epoch=1)
    torch.manual_seed(2)
    e1b = b.batches(epoch=1)
    assert e1a != plans[0] and not set(sum(e1a, [])) & set(sum(e1b, []))
    import pytest
    with pytest.raises(ValueError):
        GraphLoader(None, indices, batch_size=4, rank=0, world_size=2)  # no shared seed


def _epoch_worker(rank, world, port, q):
    """Epoch figures reduced over the ranks: rank 1 has no evaluation batch
    at all (an uneven, uncut evaluation shard)."""
    import sys

    from parity_util import PKG_ROOT
    sys.path.insert(0, PKG_ROOT)
    from vgan import dist as vdist
    from vgan.config import Configuration
    from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
    from vgan.trainer import Trainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    cfg = Configuration()
    cfg.DEVICE = "cpu"
    vdist.init("gloo", configuration=cfg)
    torch.manual_seed(cfg.SEED)
    tr = Trainer(VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12), None, None, None, None, cfg)
    if rank == 0:
        metrics = [(0.5, [0.25, 0.75], 0.4, 0.6, 0.9), (0.7, [0.5], 0.2, 0.8, 0.7)]
        losses = [[torch.tensor(1.0), torch.tensor(3.0)]]
    else:
        metrics, losses = [], [[]]
    out = tr._epoch_figures(metrics, losses)
    q.put((rank, out[0], out[1], out[2]))
    dist.destroy_process_group()


def test_gloo_epoch_figures_reduced_over_ranks():
    (_, l0, m0, lo0), (_, l1, m1, lo1) = _run(_epoch_worker)
    assert l0 == l1 == [2.0]
    assert m0 == m1
    assert m0 == pytest.approx([0.6, 0.3, 0.7, 0.8])
    assert lo0 == lo1 == 0.25


def test_eval_loader_keeps_every_batch_and_resident_replays_objects(tmp_path):
    """Evaluation loaders are not cut to a multiple of the ranks; a resident
    loader yields the same device batch objects every epoch."""
    import sys

    from parity_util import PKG_ROOT
    if PKG_ROOT not in sys.path:
        sys.path.insert(0, PKG_ROOT)
    from vgan.loader import GraphLoader
    from vgan.store import write_store
    from vgan.synth import SyntheticDataset

    indices = list(range(100, 141))  # 11 batches of 4
    a = GraphLoader(None, indices, batch_size=4, rank=0, world_size=2, seed=777, even=False)
    b = GraphLoader(None, indices, batch_size=4, rank=1, world_size=2, seed=777, even=False)
    pa, pb = a.batches(), b.batches()
    assert (len(pa), len(pb)) == (6, 5) == (len(a), len(b))
    assert sorted(i for bt in pa + pb for i in bt) == indices
    store = write_store(str(tmp_path / "st"), SyntheticDataset(6, seed=2))
    ld = GraphLoader(store, None, batch_size=4, resident=True)
    first = list(ld)
    second = list(ld)
    assert len(first) == 2 and all(x[1] is y[1] for x, y in zip(first, second))


def test_bench_launches_its_own_ranks():
    """``python bench.py --gpus 2`` with no torchrun environment starts the two
    ranks itself and relays rank 0's one JSON line; the
    CPU rehearsal (gloo, no GPU) runs the launch, the process group, the
    barriers and the max over ranks."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["VGAN_DIST_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--rehearse", "--steps", "3",
                          "--warmup", "1"], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["rehearsal"] is True
