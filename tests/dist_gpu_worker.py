"""Multi-process GPU checks for tests/test_trainer_gpu.py (run as a script).

    python tests/dist_gpu_worker.py rccl1   # one RCCL rank, sync forced on
    python tests/dist_gpu_worker.py gloo2   # two gloo ranks sharing cuda:0

Each mode prints marker lines the test reads; any failure exits non-zero.
"""
import hashlib
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _trainer(cfg, seed):
    from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
    from vgan.trainer import Trainer

    torch.manual_seed(seed)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    return Trainer(G, D, None, og, od, None, cfg)


def _digest(t):
    return hashlib.sha1(t.detach().cpu().numpy().tobytes()).hexdigest()[:16]


def rccl1():
    from vgan.config import Configuration
    from vgan.dist import GradSync
    from vgan.synth import SyntheticDataset

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    loc, vox = SyntheticDataset(16, seed=4).batch(range(4))
    loc, vox = loc.to(dev), vox.to(dev)
    ref = _trainer(cfg, 777)
    dp = _trainer(cfg, 777)
    dp.sync = GradSync(force=True)
    assert dp.sync.active and dp.sync.capturable and not ref.sync.active
    # the generator's gradient in two buckets, the decoder's reduced on a side
    # stream during the encoders' backward (RCCL AVG: no scale launch) -- an
    # opt-in (runtime['overlap_allreduce']; off by default)
    assert not dp._overlap_ready()
    cfg.runtime["overlap_allreduce"] = True
    assert dp._overlap_ready() and dp.sync.avg_op
    a = ref.step(loc, vox)  # eager: the overlap outside any capture
    b = dp.step(loc, vox)
    torch.cuda.synchronize()
    assert torch.equal(a["d_losses"], b["d_losses"]) and torch.equal(a["g_loss"], b["g_loss"])
    assert torch.equal(ref.flat_g.param, dp.flat_g.param) and torch.equal(ref.flat_d.param, dp.flat_d.param)
    for _ in range(2):
        a = ref.step_graphed(loc, vox)
        b = dp.step_graphed(loc, vox)
    torch.cuda.synchronize()
    graphs = vox.derived(dp._graph_key)
    assert graphs["sync_in_graph"] and graphs["with_adam"]
    assert torch.equal(a["d_losses"], b["d_losses"]) and torch.equal(a["g_loss"], b["g_loss"])
    assert torch.equal(ref.flat_g.param, dp.flat_g.param) and torch.equal(ref.flat_d.param, dp.flat_d.param)
    # the fresh-batch path (what Trainer.train runs at N > 1): the critic
    # iteration with its all-reduce recorded per NEW batch, the one executable
    # graph updated in place from each recording
    ds = SyntheticDataset(64, seed=8)
    for k in range(3):
        fl, fv = ds.batch(range(4 * k, 4 * k + 4))
        fl, fv = fl.to(dev), fv.to(dev)
        a = ref.step_fresh(fl, fv)
        b = dp.step_fresh(fl, fv)
        torch.cuda.synchronize()
        assert torch.equal(a["d_losses"], b["d_losses"]) and torch.equal(a["g_loss"], b["g_loss"]), k
    assert torch.equal(ref.flat_g.param, dp.flat_g.param) and torch.equal(ref.flat_d.param, dp.flat_d.param)
    # the default: the generator's gradient in one all-reduce after its
    # backward, recorded in the generator-iteration graph
    cfg.runtime["overlap_allreduce"] = False
    ref2, dp2 = _trainer(cfg, 778), _trainer(cfg, 778)
    dp2.sync = GradSync(force=True)
    assert not dp2._overlap_ready()
    for _ in range(2):
        a = ref2.step_graphed(loc, vox)
        b = dp2.step_graphed(loc, vox)
    torch.cuda.synchronize()
    assert vox.derived(dp2._graph_key)["sync_in_graph"]
    assert torch.equal(a["d_losses"], b["d_losses"]) and torch.equal(a["g_loss"], b["g_loss"])
    assert torch.equal(ref2.flat_g.param, dp2.flat_g.param) and torch.equal(ref2.flat_d.param, dp2.flat_d.param)
    dist.destroy_process_group()
    print("RCCL_GRAPH_OK", flush=True)


def _gloo_rank(rank, world, port):
    from vgan import dist as vdist
    from vgan.config import Configuration
    from vgan.synth import SyntheticDataset

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    vdist.init("gloo", configuration=cfg)
    torch.manual_seed(cfg.SEED + rank)  # bench.py's order: per-rank seed, then the models' shared seed
    ds = SyntheticDataset(64, seed=6)
    loc, vox = ds.batch([rank * 4 + i for i in range(4)])
    loc, vox = loc.to(dev), vox.to(dev)
    tr = _trainer(cfg, cfg.SEED)
    assert tr.sync.active and not tr.sync.capturable
    for _ in range(2):
        out = tr.step(loc, vox)
    out = tr.step_graphed(loc, vox)  # gloo: all-reduce + Adam eagerly between the replays
    torch.cuda.synchronize()
    print(f"RANK {rank} {_digest(tr.flat_g.param)} {_digest(tr.flat_d.param)} "
          f"{float(out['d_losses'][-1]):.9e} {tr.rng.seed}", flush=True)
    dist.destroy_process_group()


def gloo2():
    port = _free_port()
    mp.spawn(_gloo_rank, args=(2, port), nprocs=2, join=True)


if __name__ == "__main__":
    {"rccl1": rccl1, "gloo2": gloo2}[sys.argv[1]]()
