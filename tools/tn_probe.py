"""Device time of the grouped weight-gradient launch (vg_gemm_tn_group) on the
step's own product lists: one captured step records every FoldCollector
flush's products (shapes, rows per chunk), then each list is replayed on
fresh synthetic operands of the same shapes between HIP events.

    python tools/tn_probe.py [--reps 50]     # one JSON line per product list
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

# the critic's products through the Python engine's FoldCollector (the C++
# engine plans the same products with the same entry points)
os.environ.setdefault("VGAN_NATIVE_CRITIC", "0")

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--precision", default="f32")
    args = ap.parse_args()
    from vgan import _lib
    from vgan.config import Configuration

    lists = []
    orig = _lib.FoldCollector.flush

    def flush(self, stream):
        if self.products:
            lists.append([(p.N, p.M, p.K, p.rows, p.chunks, p.lda, p.ldb, p.bf16, bool(p.pdb)) for p in self.products])
        return orig(self, stream)

    _lib.FoldCollector.flush = flush
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    pool = bench.make_pool(cfg, 0, 1, 1, 32, dev)
    tr = bench.build_trainer(cfg, args.precision)
    loc, vox = pool[0]
    tr.step_graphed(loc, vox)
    torch.cuda.synchronize()
    _lib.FoldCollector.flush = orig
    seen = set()
    stream = torch.cuda.current_stream()
    for li, prods in enumerate(lists):
        key = tuple(prods)
        if key in seen:
            continue
        seen.add(key)
        keep, descs = [], []
        nbytes = flops = 0
        for (N, M, K, rows, chunks, lda, ldb, bf16, db) in prods:
            A = torch.randn(N, lda, device=dev)
            B = torch.randn(N, ldb, device=dev)
            part = torch.empty(chunks * M * K, device=dev)
            pdb = torch.empty(chunks * M, device=dev) if db else None
            keep += [A, B, part, pdb]
            d = _lib.VgTn()
            d.A, d.B, d.part = A.data_ptr(), B.data_ptr(), part.data_ptr()
            d.pdb = pdb.data_ptr() if db else None
            d.lda, d.ldb, d.N, d.M, d.K, d.rows, d.chunks, d.db_rows, d.bf16 = lda, ldb, N, M, K, rows, chunks, N, bf16
            descs.append(d)
            nbytes += 4 * N * (M + K) + 4 * chunks * M * K
            flops += 2 * N * M * K
        arr = (_lib.VgTn * len(descs))(*descs)

        def run():
            _lib.check(_lib.LIB.vg_gemm_tn_group(arr, len(descs), ctypes.c_void_p(stream.cuda_stream)),
                       "vg_gemm_tn_group")

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            run()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / args.reps
        print(json.dumps({"list": li, "products": len(prods), "us": round(us, 2), "MB": round(nbytes / 1e6, 1),
                          "GBs": round(nbytes / us / 1e3, 1), "TFLOPs": round(flops / us / 1e6, 1),
                          "shapes": [f"{p[0]}x{p[1]}x{p[2]} r{p[3]} c{p[4]}" for p in prods]}), flush=True)


if __name__ == "__main__":
    main()
