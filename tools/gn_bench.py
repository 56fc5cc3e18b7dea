"""Micro-benchmark of the GraphNorm ABI calls at the step's shapes.

    python tools/gn_bench.py [LIB.so ...]

For each library (default: the package's libvgan_hip.so), captures 20
back-to-back calls of vg_graphnorm_fwd_drop / vg_graphnorm_bwd_seg /
vg_graphnorm_jvp2 per shape in a hipGraph and reports the average device time
per call (us) from HIP events around 10 replays.  Prints one JSON line per
library."""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

from vgan import _lib  # noqa: E402

SHAPES = [(3, 12700, 64), (3, 12700, 16), (1, 12700, 64), (1, 12700, 128), (5, 12700, 8), (1, 12700, 1)]


def load(path):
    lib = ctypes.CDLL(path)
    for name in ("vg_graphnorm_seg_ws_floats", "vg_graphnorm_fwd_drop", "vg_graphnorm_bwd_seg", "vg_graphnorm_jvp2"):
        res, args = _lib.SIGNATURES[name]
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def bench(lib, dev, S, N, C, reps=20):
    P = _lib.ptr
    x = torch.randn(S * N, C, device=dev)
    w, b, ms = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3, torch.rand(C, device=dev)
    y, keep, gx, u, ju, xi = (torch.empty(S * N, C, device=dev) for _ in range(6))
    gy = torch.randn(S * N, C, device=dev)
    stats = torch.empty(S * 2 * C, device=dev)
    gw, gb, gs = (torch.zeros(C, device=dev) for _ in range(3))
    it = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(int(lib.vg_graphnorm_seg_ws_floats(S, N, C)), device=dev)

    def fwd():
        st = _lib.stream_handle(dev)
        _lib.check(lib.vg_graphnorm_fwd_drop(P(x), S, N, C, P(w), P(b), P(ms), 0.2, 7, P(it), 3, 1e-5, P(y), P(keep),
                                             P(stats), P(ws), None, st), "fwd")

    def bwd():
        st = _lib.stream_handle(dev)
        _lib.check(lib.vg_graphnorm_bwd_seg(P(x), S, N, C, P(w), P(b), P(ms), P(keep), 1e-5, P(stats), P(gy), P(gx),
                                            P(gw), P(gb), P(gs), 1, None, 0, P(ws), None, st), "bwd")

    def jvp():
        st = _lib.stream_handle(dev)
        _lib.check(lib.vg_graphnorm_jvp2(P(x), N, C, P(w), P(b), P(ms), P(keep), 1e-5, P(stats), P(u), P(gy), P(ju),
                                         P(xi), P(gw), P(gs), P(ws), None, st), "jvp2")

    out = {}
    for name, fn in (("fwd", fwd), ("bwd", bwd), ("jvp2", jvp)):
        if name == "jvp2" and S != 1:
            continue
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(e0.elapsed_time(e1) * 1e3 / (10 * reps), 2)
    return out


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    libs = sys.argv[1:] or [_lib.LIB_PATH]
    for path in libs:
        lib = load(path)
        res = {f"S{S}xN{N}xC{C}": bench(lib, dev, S, N, C) for S, N, C in SHAPES}
        print(json.dumps({"lib": os.path.basename(path), **res}), flush=True)


if __name__ == "__main__":
    main()
