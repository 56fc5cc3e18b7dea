"""BASELINE.json configs[4]: generator-only inference sweep.

    python tools/infer_sweep.py [--graphs 10000] [--batch 32] [--taus 10] [--passes 2]

Synthetic buildings (vgan.synth, seed 777) in batches of --batch; per batch one
stacked eval-mode G forward over the tau schedule 1.0 -> 0.1 (geometric, --taus
steps), f16 (vgan.half) and/or f32.  Pass 1 runs eagerly (and, graphed, captures one hipGraph per
batch); later passes replay.  Inputs are staged in HBM before timing.  Prints
one JSON line: samples/s (graphs x temperatures per second) per mode."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=10000)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--taus", type=int, default=10)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--dtype", default="f16", choices=("f16", "f32", "both"))
    args = ap.parse_args()
    from vgan.config import Configuration
    from vgan.infer import InferenceSweep, geometric_taus
    from vgan.models import VoxelGNNGenerator
    from vgan.synth import SyntheticDataset

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    G = VoxelGNNGenerator(cfg, 17, 12)
    ds = SyntheticDataset(max(args.graphs, 6500), seed=777)
    batches = []
    for b0 in range(0, args.graphs, args.batch):
        loc, vox = ds.batch(list(range(b0, min(args.graphs, b0 + args.batch))))
        batches.append((loc.to(dev), vox.to(dev)))
    taus = geometric_taus(1.0, 0.1, args.taus)
    dtypes = ("f16", "f32") if args.dtype == "both" else (args.dtype,)
    out = {"workload": f"configs[4]: {args.graphs} synthetic buildings, batch {args.batch}, "
                       f"{args.taus} Gumbel temperatures 1.0->0.1 (geometric), eval G forward",
           "unit": "samples/s (buildings x temperatures)"}
    for dt, mode in [(d, m) for d in dtypes for m in ("eager", "graphed")]:
        sw = InferenceSweep(G, taus, graphed=(mode == "graphed"), dtype=dt)
        torch.cuda.synchronize()
        times = []
        for p in range(args.passes):
            t0 = time.perf_counter()
            res = sw.run(batches)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            print(f"[infer] {dt} {mode} pass {p}: {times[-1]:.3f} s", file=sys.stderr, flush=True)
        best = min(times[1:]) if len(times) > 1 else times[0]
        out[f"{dt}_{mode}"] = {"samples_per_s": round(res["samples"] / best, 1), "pass_s": [round(t, 4) for t in times],
                     "samples_per_pass": res["samples"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
