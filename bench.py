"""Benchmark: voxel-graphs/sec of the full G+D training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N ...

Workload (BASELINE.json configs[1]): 6-type synthetic dataset, batch = 32
voxel graphs per GPU, fp32, the full step of trainer.py:466-495 (5 critic
iterations with WGAN-GP + 1 generator iteration, Adam steps included, sklearn
metrics excluded as SURVEY.md 8d specifies).  Each rank cycles over its own
pool of pre-staged batches (inputs resident in HBM when the timed region
starts); with N ranks every rank trains its own 32-building batch and the flat
gradients are averaged over RCCL (weak scaling).

Rank 0 prints ONE JSON line.  ``roofline`` is for the dominant message-passing
kernel, vg_gat_fwd: algorithmic bytes per launch / its average duration from
HIP events recorded on the launch stream around every launch of K instrumented
steps of the same workload run right after the timed region (the timed
region itself is uninstrumented).  ``roofline_stress`` is the same kernel on
config #4 (8 x 50k-node buildings, E' ~ 8.6M) where HBM, not latency, bounds it.
``cpu_baseline`` times the CPU oracle (restatement of the reference step,
pinned bit-for-bit to the reference by tests/golden) on one batch-32 step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd")
for _p in (ROOT, PKG_ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "voxel-graphs/sec (full G+D step)"


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def gat_fwd_bytes(n: int, e: int, c: int) -> int:
    """Algorithmic bytes of one vg_gat_fwd: read h [N,C], write out [N,C],
    read row_ptr [N+1] and col [E'], write alpha [E'] and a_src/a_dst [N],
    read att_src/att_dst/bias [C]."""
    return 4 * (2 * n * c + (n + 1) + 2 * e + 2 * n + 3 * c)


class GatTimer:
    """HIP-event timing of every vg_gat_fwd launch (on its launch stream)."""

    def __init__(self):
        self.records = []

    def install(self):
        from vgan import ops

        orig = ops._GATConv.forward
        timer = self

        def timed_forward(ctx, h, att_src, att_dst, bias, csr, slope):
            stream = torch.cuda.current_stream(h.device)
            start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            start.record(stream)
            out = orig(ctx, h, att_src, att_dst, bias, csr, slope)
            end.record(stream)
            timer.records.append((start, end, gat_fwd_bytes(csr.num_nodes, csr.num_edges, h.shape[1])))
            return out

        self._orig = orig
        ops._GATConv.forward = staticmethod(timed_forward)

    def uninstall(self):
        from vgan import ops

        ops._GATConv.forward = staticmethod(self._orig)

    def summary(self):
        torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e, _ in self.records]
        nbytes = [b for _, _, b in self.records]
        n = len(ms)
        avg_ms = sum(ms) / n
        avg_bytes = sum(nbytes) / n
        achieved = avg_bytes / (avg_ms * 1e-3) / 1e9
        return {"launches": n, "avg_us": avg_ms * 1e3, "avg_bytes": avg_bytes, "achieved_gbs": achieved}


def make_pool(cfg, rank: int, world: int, pool: int, batch: int, device):
    from vgan.synth import SyntheticDataset

    ds = SyntheticDataset(6500, seed=777)
    out = []
    for b in range(pool):
        idx = [((b * world + rank) * batch + i) % len(ds) for i in range(batch)]
        loc, vox = ds.batch(idx)
        out.append((loc.to(device), vox.to(device)))
    return out


def build_trainer(cfg):
    from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
    from vgan.trainer import Trainer

    torch.manual_seed(cfg.SEED)
    G = VoxelGNNGenerator(cfg, 17, 12)
    D = VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(og, T_max=cfg.EPOCHS)
    return Trainer(G, D, None, og, od, sched, cfg)


GRAPHED = True


def run_steps(tr, pool, k: int, offset: int = 0):
    out = None
    for s in range(k):
        loc, vox = pool[(offset + s) % len(pool)]
        out = tr.step_graphed(loc, vox) if GRAPHED else tr.step(loc, vox)
    return out


def stress_roofline(device, channels=(128, 64, 1), reps: int = 20):
    from vgan import ops
    from vgan.synth import make_stress_building
    from vgan.graph import GraphBatch

    items = [make_stress_building(777, i) for i in range(8)]
    vox = GraphBatch.from_data_list([v for _, v in items]).to(device)
    csr = ops.CSR(vox.edge_index, vox.num_nodes)
    n, e = csr.num_nodes, csr.num_edges
    scratch = torch.empty(512 * 1024 * 1024 // 4, device=device)  # flush the 256 MB MALL between reps
    res = {}
    for c in channels:
        h = torch.randn(n, c, device=device)
        att_s, att_d = torch.randn(c, device=device) * 0.1, torch.randn(c, device=device) * 0.1
        bias = torch.randn(c, device=device)
        with torch.no_grad():
            for _ in range(3):
                ops.gat_conv(csr, h, att_s, att_d, bias)
            times = []
            for _ in range(reps):
                scratch.fill_(1.0)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                ops.gat_conv(csr, h, att_s, att_d, bias)
                en.record()
                torch.cuda.synchronize()
                times.append(st.elapsed_time(en))
        avg = sum(times) / len(times)
        b = gat_fwd_bytes(n, e, c)
        res[c] = {"avg_us": avg * 1e3, "bytes": b, "achieved_gbs": b / (avg * 1e-3) / 1e9}
    del scratch
    return {"nodes": n, "edges": e, "per_channels": res}


def cpu_baseline(cfg_batch: int, seconds_budget: float):
    """Time the CPU oracle (reference step restatement) on a batch-32 step."""
    from oracle import pyg
    from oracle import reference as R
    from vgan.config import Configuration
    from vgan.synth import SyntheticDataset

    threads = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if cap > 0:
        threads = min(threads, cap)
    torch.set_num_threads(threads)
    cfg = Configuration()
    ds = SyntheticDataset(6500, seed=777)
    items = [ds[i] for i in range(cfg_batch)]
    keys_v = ("x", "edge_index", "type", "types_onehot", "site_area", "data_number")
    keys_l = ("x", "type", "data_number")
    local = pyg.Batch.from_data_list([pyg.Data(**{k: getattr(l, k) for k in keys_l}) for l, _ in items])
    voxel = pyg.Batch.from_data_list([pyg.Data(**{k: getattr(v, k) for k in keys_v}) for _, v in items])
    torch.manual_seed(777)
    G, D = R.Generator(cfg), R.Discriminator(cfg)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    steps, t_total = 0, 0.0
    while True:
        t0 = time.perf_counter()
        R.train_step(G, D, og, od, cfg, local, voxel)
        t_total += time.perf_counter() - t0
        steps += 1
        log(f"cpu baseline step {steps}: {t_total / steps:.2f} s/step")
        if t_total >= seconds_budget * 0.5 or steps >= 3:
            break
    return {
        "value": round(cfg_batch * steps / t_total, 3),
        "unit": "graphs/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "sample": f"{steps} full G+D step(s) of batch {cfg_batch} synthetic buildings "
                  f"({voxel.num_nodes} voxel nodes) through the CPU oracle (oracle/reference.py, "
                  f"pinned bit-for-bit to the reference's own trainer.py step), fp32, "
                  f"{t_total / steps:.2f} s/step",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--pool", type=int, default=4, help="pre-staged batches per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-stress", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture of the step")
    ap.add_argument("--profile", action="store_true",
                    help="for rocprofv3: only warm-up + timed steps (50 ms idle gap before the timed region), "
                         "no instrumented / stress / CPU passes")
    args = ap.parse_args()
    global GRAPHED
    GRAPHED = not args.eager

    rank, world, local = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(
        os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)

    from vgan.config import Configuration

    cfg = Configuration()
    cfg.DEVICE = str(device)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED + rank)
    torch.cuda.manual_seed(cfg.SEED + rank)
    log(f"rank {rank}/{world}: staging {args.pool} batches of {args.batch} buildings")
    pool = make_pool(cfg, rank, world, args.pool, args.batch, device)
    tr = build_trainer(cfg)
    n_nodes = sum(v.num_nodes for _, v in pool) / len(pool)

    # warm-up (also builds every batch's CSR / type-mean once, as the first step of a batch would)
    for (loc, vox) in pool:
        run_steps(tr, [(loc, vox)], 1)
    run_steps(tr, pool, args.warmup)
    torch.cuda.synchronize()
    log("warm-up done")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if args.profile:
        time.sleep(0.05)  # idle gap that tools/prof_summary.py --after-gap keys on
    t0 = time.perf_counter()
    for s in range(args.steps):
        run_steps(tr, pool, 1, offset=s)
        if (s + 1) % 10 == 0:
            log(f"step {s + 1}/{args.steps}")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = args.batch * world * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    log(f"timed ({'hipGraph' if GRAPHED else 'eager'}): {ms_per_step:.2f} ms/step, {value:.1f} graphs/s")

    if args.profile:
        if rank == 0:
            print(json.dumps({"profile": True, "value": round(value, 3), "ms_per_step": round(ms_per_step, 3),
                              "steps": args.steps}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # instrumented pass for the dominant kernel's roofline (eager: per-launch
    # HIP events around vg_gat_fwd on its launch stream)
    timer = GatTimer()
    timer.install()
    GRAPHED, was = False, GRAPHED
    run_steps(tr, pool, args.steps)
    GRAPHED = was
    timer.uninstall()
    kern = timer.summary()
    log(f"vg_gat_fwd: {kern['launches']} launches, avg {kern['avg_us']:.2f} us, {kern['achieved_gbs']:.1f} GB/s")

    result = None
    if rank == 0:
        stress = None if args.no_stress else stress_roofline(device)
        if stress:
            for c, r in stress["per_channels"].items():
                log(f"stress C={c}: {r['avg_us']:.1f} us, {r['achieved_gbs']:.0f} GB/s")
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.batch, args.cpu_seconds)
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "graphs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded 6-type buildings in the reference tensor layout; random-init weights)",
            "config": {
                "workload": "configs[1]: 6-type dataset, batch=32 voxel graphs per GPU, fp32, full G+D step "
                            "(5 critic WGAN-GP + 1 generator iteration, Adam), HIP message passing",
                "global_batch": args.batch * world,
                "avg_voxel_nodes_per_batch": round(n_nodes, 1),
                "parallelism": f"dp{world}",
                "execution": ("hipGraph replay: one stacked no-grad G forward for the N_CRITIC critic labels, "
                              "N_CRITIC critic-engine graphs, one generator-iteration graph") if GRAPHED else "eager",
            },
            "roofline": {
                "kernel": "vg_gat_fwd (fused GAT edge softmax + CSR gather-sum)",
                "bound": "hbm",
                "achieved": round(kern["achieved_gbs"], 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(kern["achieved_gbs"] / HBM_PEAK_GBS, 5),
                "traffic": None,
                "avg_launch_us": round(kern["avg_us"], 3),
                "avg_algorithmic_bytes": int(kern["avg_bytes"]),
                "launches_timed": kern["launches"],
            },
            "cpu_baseline": cpu,
        }
        if stress:
            c128 = stress["per_channels"][128]
            result["roofline_stress"] = {
                "workload": f"configs[3]: 8 x 50k-node buildings, N={stress['nodes']}, E'={stress['edges']}, "
                            "C=128 fp32, cold MALL",
                "bound": "hbm", "achieved": round(c128["achieved_gbs"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(c128["achieved_gbs"] / HBM_PEAK_GBS, 4), "avg_launch_us": round(c128["avg_us"], 2),
                "per_channels": {str(c): {k: round(v, 2) for k, v in r.items()}
                                 for c, r in stress["per_channels"].items()},
            }
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
