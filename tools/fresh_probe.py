"""Where the fresh-batch step loses time against the replayed step.

    python tools/fresh_probe.py [--steps 40] [--warmup 5]

Variants of bench.py's fresh-batch leg (a NEW batch every step through
Trainer._train_batch -> step_fresh), each timed between device syncs:

  loader    GraphLoader prefetching 3 batches on its thread (bench.py's leg)
  staged    the same batches collated and uploaded before the timed region
            (each batch still new to the trainer: CSR adopt, type-mean, ELL,
            capture inside the timed region)
  switch    loader, with sys.setswitchinterval(1e-4) (GIL hand-off)
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402


def run(variant, cfg, bench, dev, steps, warmup, batch=32):
    from vgan.loader import GraphLoader
    from vgan.store import write_store
    from vgan.synth import SyntheticDataset

    n = warmup + steps
    tmp = tempfile.mkdtemp(prefix="vgan_probe_")
    ds = SyntheticDataset(n * batch, seed=4321)
    store = write_store(os.path.join(tmp, "store"), ds)
    loader = GraphLoader(store, batch_size=batch, shuffle=True, device=dev, prefetch=3, seed=4321)
    torch.manual_seed(cfg.SEED)
    tr = bench.build_trainer(cfg, "f32")
    cfg.runtime["train_step"] = "auto"
    old = sys.getswitchinterval()
    if variant == "switch":
        sys.setswitchinterval(1e-4)
    if variant == "staged":
        batches = list(loader)
        torch.cuda.synchronize()
        it = iter(batches)
    else:
        it = iter(loader)
    for _ in range(warmup):
        tr._train_batch(*next(it))
    torch.cuda.synchronize()
    per = []
    t0 = time.perf_counter()
    for _ in range(steps):
        a = time.perf_counter()
        tr._train_batch(*next(it))
        per.append((time.perf_counter() - a) * 1e3)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps * 1e3
    sys.setswitchinterval(old)
    del it, loader
    shutil.rmtree(tmp, ignore_errors=True)
    per.sort()
    return {"variant": variant, "ms_per_step": round(el, 3), "host_call_ms_median": round(per[len(per) // 2], 3),
            "host_call_ms_max": round(per[-1], 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--variants", default="loader,staged,switch,loader")
    args = ap.parse_args()
    import bench
    from vgan.config import Configuration

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    for v in args.variants.split(","):
        print(json.dumps(run(v, cfg, bench, dev, args.steps, args.warmup)), flush=True)


if __name__ == "__main__":
    main()
