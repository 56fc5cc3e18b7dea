"""Per-launch device time of the aggregation (vg_gat_aggregate_fwd, with and
without the GraphNorm partials) against graph size: is a launch of the step
bound by its rows' latency chain (time flat in N) or by throughput (time
growing with N)?  Each point: 50 identical launches captured in one hipGraph,
replayed between HIP events.  A streaming copy of the same h/out bytes is
timed beside it.  One JSON line per point.

    python tools/agg_latency_probe.py
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402


def timed(fn, k=50, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(k):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (k * reps)


def main():
    from vgan import data as vdata
    from vgan import ops
    from vgan._lib import ptr, stream_handle
    from vgan.synth import SyntheticDataset

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ds = SyntheticDataset(64, seed=777)
    one = torch.zeros(1, device=dev)
    print(json.dumps({"tiny_add_us": round(timed(lambda: one.add_(1.0)), 2)}), flush=True)
    for nb, copies in ((1, 1), (4, 1), (16, 1), (32, 1), (32, 3), (32, 5)):
        loc, vox = ds.batch(range(nb))
        loc, vox = loc.to(dev), vox.to(dev)
        csr = vdata.prepared(loc, vox, 12).csr.stacked(copies)
        n = csr.num_nodes
        for c in (1, 8, 32, 64):
            h = torch.randn(n, c, device=dev)
            a_s, a_d = 0.3 * torch.randn(n, device=dev), 0.3 * torch.randn(n, device=dev)
            b = torch.randn(c, device=dev)
            out, alpha = torch.empty_like(h), torch.empty(csr.num_edges, device=dev)
            part = ops.gnp_buffer(csr, c, dev)[0]
            def agg(gnp=None):  # on the current (capturing) stream
                ops.aggregate_fwd_raw(csr, c, ptr(h), ptr(a_s), ptr(a_d), ptr(b), 0.2, ptr(out), ptr(alpha),
                                      stream_handle(dev), gnp)

            y = torch.empty_like(h)
            rec = {"buildings": nb, "copies": copies, "rows": n, "edges": csr.num_edges, "C": c,
                   "plain_us": round(timed(agg), 2), "gnp_us": round(timed(lambda: agg(part)), 2),
                   "copy_us": round(timed(lambda: y.copy_(h)), 2)}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
