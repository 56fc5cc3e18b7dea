"""Device time of the deferred-fold launches (vg_fold_batch) on the step's own
fold lists: one captured step records every vg_fold_batch call (each fold's
width, partial rows per source), then each list is replayed on fresh
synthetic partials between HIP events -- whole, and fold by fold (which fold
is the launch's long pole).

    python tools/fold_probe.py [--reps 50]     # one JSON line per fold list
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))
# the critic's folds through the Python engine's FoldCollector (the C++
# engine batches the same folds the same way)
os.environ.setdefault("VGAN_NATIVE_CRITIC", "0")

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    from vgan import _lib
    from vgan.config import Configuration

    lists = []
    orig = _lib.LIB.vg_fold_batch

    class Spy:
        def __call__(self, arr, n, stream):
            lists.append([(arr[i].width, arr[i].k, arr[i].nsrc, [(arr[i].src[s].rows, arr[i].src[s].ld)
                                                                   for s in range(arr[i].nsrc)])
                          for i in range(int(n))])
            return orig(arr, n, stream)

    _lib.LIB.vg_fold_batch = Spy()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    pool = bench.make_pool(cfg, 0, 1, 1, 32, dev)
    tr = bench.build_trainer(cfg, "f32")
    loc, vox = pool[0]
    tr.step_graphed(loc, vox)
    torch.cuda.synchronize()
    _lib.LIB.vg_fold_batch = orig
    stream = torch.cuda.current_stream()
    seen = set()

    def timed(descs):
        arr = (_lib.VgFold * len(descs))(*descs)

        def run():
            _lib.check(orig(arr, len(descs), ctypes.c_void_p(stream.cuda_stream)), "vg_fold_batch")

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            run()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / args.reps

    for li, folds in enumerate(lists):
        key = repr(folds)
        if key in seen:
            continue
        seen.add(key)
        keep, descs = [], []
        nbytes = 0
        for (width, k, nsrc, srcs) in folds:
            d = _lib.VgFold()
            out = torch.zeros(width, device=dev)
            keep.append(out)
            d.out, d.width, d.k, d.ldo, d.accumulate, d.nsrc = out.data_ptr(), width, k, k, 1, nsrc
            for s, (rows, ld) in enumerate(srcs):
                p = torch.randn(max(1, rows * ld), device=dev)
                keep.append(p)
                d.src[s].part, d.src[s].rows, d.src[s].ld = p.data_ptr(), rows, ld
                nbytes += 4 * rows * width
            descs.append(d)
        us = timed(descs)
        each = [round(timed([d]), 2) for d in descs]
        print(json.dumps({"list": li, "folds": len(folds), "us": round(us, 2), "MB": round(nbytes / 1e6, 2),
                          "GBs": round(nbytes / us / 1e3, 1),
                          "folds_wxrows_us": [f"{f[0]}x{'+'.join(str(r) for r, _ in f[3])}:{t}"
                                              for f, t in zip(folds, each)]}), flush=True)


if __name__ == "__main__":
    main()
