"""Per-shape device time of the Linear + LayerNorm + LeakyReLU GEMM
(vg_gemm_ln_act via vgan.nn.linear_ln_act) and the plain GEMM (vgan.nn.linear)
at the step's row counts, no-grad (the forward kernel only).

    python tools/ln_gemm_probe.py [f32|bf16]   # one JSON line per shape
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "building-gan-graph-conditioned-architectural-volume-generation_amd"))
from vgan._lib import gemm_precision_scope  # noqa: E402
from vgan.nn import linear, linear_ln_act  # noqa: E402


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    prec = sys.argv[1] if len(sys.argv) > 1 else "f32"
    only = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else None  # rows,K,M: that shape only
    shapes = [(n, k, m) for n in (12700, 38100, 63500)
              for k, m in ((17, 128), (128, 128), (268, 128), (524, 128), (128, 64), (36, 64), (64, 64))]
    for n, k, m in ([tuple(only)] if only else shapes):
        x = torch.randn(n, k, device=dev)
        w = torch.randn(m, k, device=dev) / k ** 0.5
        b = torch.randn(m, device=dev)
        g, be = torch.ones(m, device=dev), torch.zeros(m, device=dev)
        with torch.no_grad(), gemm_precision_scope(prec):
            t_ln = timed(lambda: linear_ln_act(x, w, b, g, be)) if m > 64 or True else None
            t_lin = timed(lambda: linear(x, w, b))
        fl = 2.0 * n * k * m
        print(json.dumps({"precision": prec, "rows": n, "K": k, "M": m, "ln_us": round(t_ln, 2), "linear_us": round(t_lin, 2),
                          "ln_tflops": round(fl / t_ln / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
