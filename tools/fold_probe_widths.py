"""Device time of single deferred-gradient folds (vg_fold_batch with one
fold) by shape, graph-replayed between HIP events: partial rows x width as
the critic iteration and the generator backward produce them (GAT parameter
partials per 32-row workgroup of a 38k-row stacked backward, split-K
weight-gradient partials).  Finds the long pole of the fold launch.

    python tools/fold_probe_widths.py     # JSON lines
    FOLD_COLD=1 ...                       # the partials rewritten before each fold (the rewrite's own time subtracted)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

from vgan._lib import LIB, VgFold, VgFoldSrc, check, stream_handle  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = stream_handle(dev)
    shapes = [(1191, w) for w in (4, 8, 16, 32, 64, 128, 256)] + [(398, w) for w in (32, 128)] + \
             [(256, w) for w in (256, 1024, 4096, 16384)] + [(64, 16384), (32, 67072)]
    for rows, width in shapes:
        part = torch.randn(rows, width, device=dev)
        out = torch.zeros(width, device=dev)
        f = VgFold()
        f.out, f.width, f.k, f.ldo, f.accumulate, f.nsrc = out.data_ptr(), width, width, width, 1, 1
        f.src[0] = VgFoldSrc(part.data_ptr(), rows, width)
        arr = (VgFold * 1)(f)

        def run():
            check(LIB.vg_fold_batch(arr, 1, st), "vg_fold_batch")

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        cold = os.environ.get("FOLD_COLD", "0") == "1"
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(20):
                    if cold:  # the partials rewritten just before, as a producing kernel leaves them
                        part.mul_(1.0)
                    check(LIB.vg_fold_batch(arr, 1, stream_handle(dev)), "vg_fold_batch")
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        if cold:  # minus the rewrite alone
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g2, stream=s):
                    for _ in range(20):
                        part.mul_(1.0)
            g2.replay()
            torch.cuda.synchronize()
            a2, b2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a2.record()
            g2.replay()
            b2.record()
            torch.cuda.synchronize()
            base = a2.elapsed_time(b2) * 1e3 / 20
        else:
            base = 0.0
        print(json.dumps({"rows": rows, "width": width, "cold": cold,
                          "us": round(a.elapsed_time(b) * 1e3 / 20 - base, 2)}), flush=True)


if __name__ == "__main__":
    main()
