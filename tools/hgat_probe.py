"""Per-width device time of the f16 aggregation (vg_hgat_fwd) at the configs[4]
sweep's shapes: a batch of 32 buildings stacked over the 10 Gumbel
temperatures (~121k rows), one launch per encoder width, 50 identical launches
captured in one hipGraph and replayed between HIP events.  One JSON line per
width: us per launch and algorithmic GB/s (bench.py agg_bytes, f16 rows).

    python tools/hgat_probe.py
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
    from bench import agg_bytes
    from vgan import data as vdata
    from vgan._lib import LIB, check, ptr, stream_handle
    from vgan.synth import SyntheticDataset

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    loc, vox = SyntheticDataset(64, seed=777).batch(range(32))
    loc, vox = loc.to(dev), vox.to(dev)
    copies = int(os.environ.get("HGAT_COPIES", "10"))
    csr = vdata.prepared(loc, vox, 7).csr.stacked(copies)
    rows, e = csr.num_nodes, csr.num_edges
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    for c in (1, 2, 4, 8, 16, 32, 64, 128):
        ld = (c + 7) // 8 * 8
        h = (torch.randn(rows, ld, device=dev, generator=gen) * 0.5).half()
        a_s = 0.3 * torch.randn(rows, device=dev, generator=gen)
        a_d = 0.3 * torch.randn(rows, device=dev, generator=gen)
        bias = torch.randn(c, device=dev, generator=gen)
        o = torch.empty(rows, ld, dtype=torch.float16, device=dev)

        def run():
            check(LIB.vg_hgat_fwd(ptr(csr.row_ptr), ptr(csr.col), rows, c, ld, ptr(h), ptr(a_s), ptr(a_d), ptr(bias),
                                  0.2, ptr(o), ld, stream_handle(dev)), "vg_hgat_fwd")

        us = timed(run)
        b = agg_bytes(rows, e, c, elem=2)
        rec = {"C": c, "ld": ld, "rows": rows, "edges": e, "us": round(us, 2), "algorithmic_bytes": b,
               "gbs": round(b / (us * 1e-6) / 1e9, 1)}
        if os.environ.get("HGAT_GN") == "1":  # the block's aggregation + GraphNorm, with / without the partials
            n = rows // copies
            g = int(LIB.vg_hgat_gnp_rows(rows, ld))
            gnp = torch.empty(max(1, int(LIB.vg_hgat_gnp_floats(rows, ld))), device=dev)
            w, bb, ms = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev), torch.rand(c, device=dev)
            y = torch.empty_like(o)
            stats = torch.empty(copies * 2 * c, device=dev)
            ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(copies, n, c)), device=dev)

            def run_gnp():
                check(LIB.vg_hgat_fwd_gnp(ptr(csr.row_ptr), ptr(csr.col), rows, c, ld, ptr(h), ptr(a_s), ptr(a_d),
                                          ptr(bias), 0.2, ptr(o), ld, n, ptr(gnp), stream_handle(dev)), "gnp")

            def pair_old():
                run()
                check(LIB.vg_graphnorm_fwd_h(ptr(o), ld, copies, n, c, ptr(w), ptr(bb), ptr(ms), 1e-5, ptr(y), ld,
                                             ptr(stats), ptr(ws), stream_handle(dev)), "gn")

            def pair_new():
                run_gnp()
                check(LIB.vg_graphnorm_fwd_h_gnp(ptr(o), ld, copies, n, c, ptr(w), ptr(bb), ptr(ms), 1e-5, ptr(y), ld,
                                                 ptr(stats), ptr(gnp), g, stream_handle(dev)), "gn_gnp")

            rec.update({"gnp_us": round(timed(run_gnp), 2), "block_stats_pass_us": round(timed(pair_old), 2),
                        "block_partials_us": round(timed(pair_new), 2)})
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
