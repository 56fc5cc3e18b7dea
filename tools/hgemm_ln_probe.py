"""Device time of the f16 LayerNorm GEMM (vg_hgemm_ln_act, M = 128) at the
configs[4] sweep's shapes: 131k stacked rows (10 temperatures x a batch of 32
buildings), K = 128 (the MLP encoder's inner layers), 272 (its first layer,
268 padded) and 528 (the decoder's first, 524 padded); and 13k rows (the
program-feature encoder, run once per batch).  50 identical launches in one
hipGraph, replayed between HIP events; a device copy of the same bytes
(A in + Y out) beside each.  One JSON line per shape.

    python tools/hgemm_ln_probe.py
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from agg_latency_probe import timed  # noqa: E402


def main():
    from vgan._lib import LIB, check, ptr, stream_handle

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    for n, k in ((131070, 128), (131070, 272), (131070, 528), (13107, 128)):
        m = 128
        a = (torch.randn(n, k, device=dev, generator=g) * 0.5).half()
        w = (torch.randn(m, k, device=dev, generator=g) * 0.1).half()
        b, gam, bet = torch.randn(m, device=dev), torch.rand(m, device=dev) + 0.5, torch.randn(m, device=dev)
        y = torch.empty(n, m, dtype=torch.float16, device=dev)

        def run():
            check(LIB.vg_hgemm_ln_act(ptr(a), k, ptr(w), k, n, m, k, ptr(b), ptr(gam), ptr(bet), 1e-5, 0.2, ptr(y), m,
                                      stream_handle(dev)), "vg_hgemm_ln_act")

        def run_bias():  # the same GEMM with the bias + LeakyReLU epilogue (no LayerNorm)
            check(LIB.vg_hgemm(ptr(a), k, ptr(w), k, n, m, k, ptr(b), 2, 0.2, ptr(y), m, 0, stream_handle(dev)),
                  "vg_hgemm")

        src = torch.empty(n * (k + m), dtype=torch.float16, device=dev)
        dst = torch.empty_like(src)
        us = timed(run)
        cu = timed(lambda: dst.copy_(src))
        byts = 2 * n * (k + m)
        print(json.dumps({"rows": n, "K": k, "M": m, "us": round(us, 2), "gbs": round(byts / (us * 1e-6) / 1e9, 1),
                          "copy_same_bytes_us": round(cu / 2, 2), "no_ln_us": round(timed(run_bias), 2), "tflops": round(2 * n * m * k / (us * 1e-6) / 1e12, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
