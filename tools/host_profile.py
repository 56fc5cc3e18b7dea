"""Host-side cost of the eager step (the path a fresh batch takes).

    python tools/host_profile.py [--steps 10] [--sort tottime]

Builds the bench's trainer on one batch of 32 buildings and times, host-side
only (no synchronisation inside the measured region), each phase of the eager
step -- the stacked critic-label forward, one critic iteration, the generator
iteration -- then runs cProfile over whole eager steps and prints the top
functions.  The device time of the same step is ~8 ms (bench.py); whatever the
host needs beyond that is what a fresh batch pays.
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--sort", default="tottime")
    ap.add_argument("--fresh", action="store_true",
                    help="profile step_fresh (the fresh-batch path) over distinct staged batches")
    ap.add_argument("--top", type=int, default=45)
    args = ap.parse_args()
    import bench

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from vgan.config import Configuration

    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    pool = bench.make_pool(cfg, 0, 1, 1, 32, dev)
    tr = bench.build_trainer(cfg, "f32")
    if args.fresh:
        return fresh(args, cfg, tr, bench, dev)
    loc, vox = pool[0]
    for _ in range(3):
        tr.step(loc, vox)
    torch.cuda.synchronize()
    # host time per phase (the device runs behind; no sync inside)
    phases = {"labels": [], "critic": [], "gen": [], "step": []}
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        labels = tr._critic_labels(loc, vox)
        t1 = time.perf_counter()
        for i in range(cfg.N_CRITIC):
            tr._critic_iteration(loc, vox, labels, i)
            tr.adam_d.step(counted=True)
        t2 = time.perf_counter()
        tr._gen_iteration(loc, vox)
        tr.adam_g.step(counted=True)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        phases["labels"].append(t1 - t0)
        phases["critic"].append((t2 - t1) / cfg.N_CRITIC)
        phases["gen"].append(t3 - t2)
        phases["step"].append(t4 - t0)
    for k, v in phases.items():
        v = sorted(v)
        print(f"host {k:7s}: median {v[len(v) // 2] * 1e3:7.3f} ms" + (" (per critic iteration)" if k == "critic" else
                                                                       " (incl. device drain)" if k == "step" else ""))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        tr.step(loc, vox)
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(args.sort).print_stats(args.top)
    print(s.getvalue())


def fresh(args, cfg, tr, bench, dev):
    """Host time per phase of step_fresh (marks from Trainer.phase_hook), the
    device drained only between steps, then cProfile over whole steps."""
    pool = bench.make_pool(cfg, 0, 1, 8, 32, dev)
    for k in range(3):
        tr.step_fresh(*pool[k % len(pool)])
    torch.cuda.synchronize()
    times = {}
    last = [0.0]

    def mark(name):
        now = time.perf_counter()
        times.setdefault(name, []).append(now - last[0])
        last[0] = now

    tr.phase_hook = mark
    totals = []
    for k in range(args.steps):
        torch.cuda.synchronize()
        t0 = last[0] = time.perf_counter()
        tr.step_fresh(*pool[k % len(pool)])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        totals.append((t1 - t0, time.perf_counter() - t0))
    tr.phase_hook = None
    for name, v in times.items():
        v = sorted(v)
        print(f"host {name:8s}: median {v[len(v) // 2] * 1e3:7.3f} ms")
    enq = sorted(t for t, _ in totals)
    full = sorted(t for _, t in totals)
    print(f"host enqueue total: median {enq[len(enq) // 2] * 1e3:7.3f} ms; with device drain {full[len(full) // 2] * 1e3:7.3f} ms")
    # back-to-back steps (no drain between): the rate the fresh-batch leg sees
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        tr.step_fresh(*pool[k % len(pool)])
    torch.cuda.synchronize()
    print(f"back-to-back step_fresh: {(time.perf_counter() - t0) / args.steps * 1e3:.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for k in range(args.steps):
        tr.step_fresh(*pool[k % len(pool)])
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(args.sort).print_stats(args.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
