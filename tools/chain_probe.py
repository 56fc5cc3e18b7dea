"""vg_linear_chain vs the per-layer vg_gemm launches it replaces, graph-replayed
between HIP events at the critic's shapes (R = 3N = 38k rows forward / adjoint,
N = 12.7k rows tangent).  One JSON line.

    python tools/chain_probe.py [--rows 38100] [--reps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402


def timed(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=38100)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    from vgan import _lib
    from vgan._lib import LIB, check, ptr, stream_handle

    dev = torch.device("cuda", 0)
    res = {}
    for case, widths, wt, acts, rows in (("forward", [64, 32, 16, 8, 1], 0, [1, 1, 1, 0], args.rows),
                                         ("tangent", [64, 32, 16, 8], 0, [3, 3, 3], args.rows // 3),
                                         ("adjoint", [1, 8, 16, 32], 1, [3, 3, 3], args.rows)):
        x = torch.randn(rows, widths[0], device=dev)
        Ws, bs, auxs, outs = [], [], [], []
        for i in range(len(widths) - 1):
            a, b = widths[i], widths[i + 1]
            Ws.append(torch.randn(*((b, a) if not wt else (a, b)), device=dev))
            bs.append(torch.randn(b, device=dev) if case == "forward" else None)
            auxs.append(torch.randn(rows, b, device=dev))
            outs.append(torch.empty(rows, b, device=dev))
        layers = [dict(weight=Ws[i].data_ptr(), bias=bs[i].data_ptr() if bs[i] is not None else None,
                       aux=auxs[i].data_ptr(), ld_aux=widths[i + 1], out=outs[i].data_ptr(), ld_out=widths[i + 1],
                       w_trans=wt, act=acts[i]) for i in range(len(widths) - 1)]

        def chain():
            assert _lib.linear_chain(ptr(x), widths[0], rows, widths, layers, stream_handle(dev))

        def gemms():
            st = stream_handle(dev)
            inp, k = x, widths[0]
            for i in range(len(widths) - 1):
                m = widths[i + 1]
                if wt:  # C = A W, W [k][m]
                    check(LIB.vg_gemm(ptr(inp), k, ptr(Ws[i]), m, 0, None, acts[i], ptr(auxs[i]), m, ptr(outs[i]), m,
                                      rows, m, k, st), "gemm")
                else:
                    check(LIB.vg_gemm(ptr(inp), k, ptr(Ws[i]), k, 1, ptr(bs[i]), acts[i], ptr(auxs[i]), m,
                                      ptr(outs[i]), m, rows, m, k, st), "gemm")
                inp, k = outs[i], m

        res[case] = {"rows": rows, "chain_us": round(timed(chain, args.reps), 2),
                     "gemms_us": round(timed(gemms, args.reps), 2), "layers": len(widths) - 1}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
