"""Aggregate-then-project probe (verdict r05 item 4(c)): for GATConv's
widening layers, out = A (X W^T) + b = (A X) W^T + b, with A the attention
matrix, whose logits need only a_s = X (W^T att_src) and a_d = X (W^T att_dst).
So the aggregation can run at Cin channels and the projection follow it.  Per
widening block (Cin -> Cout) at the step's shapes (batch 32, one copy and the
critic's three stacked copies), the device time of

  project-then-aggregate (the shipped form): vg_gat_lin_att (GEMM + the a_s /
      a_d epilogue) -> vg_gat_aggregate_fwd_gnp at Cout (with the GraphNorm
      partials)
  aggregate-then-project: a_s / a_d as one [2, N] product X (W^T att)^T
      (vg_gemm, 2 rows) -> vg_gat_aggregate_fwd at Cin -> vg_gemm (A X) W^T + b
      at Cout (no GraphNorm partials: they would need an epilogue this GEMM
      does not have, so this form is timed with less work than it would do)

each as 50 identical sequences captured in one hipGraph, replayed between HIP
events.  One JSON line per point.

    python tools/agg_project_probe.py
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from agg_latency_probe import timed  # noqa: E402


def main():
    from vgan import data as vdata
    from vgan import ops
    from vgan._lib import LIB, check, ptr, stream_handle
    from vgan.synth import SyntheticDataset

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ds = SyntheticDataset(64, seed=777)
    loc, vox = ds.batch(range(32))
    loc, vox = loc.to(dev), vox.to(dev)
    base = vdata.prepared(loc, vox, 12).csr
    torch.manual_seed(0)
    for copies in (1, 3):
        csr = base.stacked(copies) if copies > 1 else base
        n = csr.num_nodes
        for cin, cout in ((8, 16), (16, 32), (32, 64), (64, 128)):
            x = torch.randn(n, cin, device=dev)
            w = torch.randn(cout, cin, device=dev) / cin ** 0.5
            att_s, att_d = torch.randn(cout, device=dev) * 0.1, torch.randn(cout, device=dev) * 0.1
            bias = torch.randn(cout, device=dev)
            zero_b = torch.zeros(cin, device=dev)
            w_att = torch.stack([w.t() @ att_s, w.t() @ att_d]).contiguous()  # [2, cin]
            h = torch.empty(n, cout, device=dev)
            a_s, a_d = torch.empty(n, device=dev), torch.empty(n, device=dev)
            out = torch.empty(n, cout, device=dev)
            alpha = torch.empty(csr.num_edges, device=dev)
            gnp, _ = ops.gnp_buffer(csr, cout, dev)
            sd = torch.empty(2, n, device=dev)
            z = torch.empty(n, cin, device=dev)

            def project_then_aggregate():
                st = stream_handle(dev)  # the current (capturing) stream
                check(LIB.vg_gat_lin_att(ptr(x), cin, ptr(w), n, cin, cout, ptr(att_s), ptr(att_d), ptr(h), ptr(a_s),
                                         ptr(a_d), st), "vg_gat_lin_att")
                ops.aggregate_fwd_raw(csr, cout, ptr(h), ptr(a_s), ptr(a_d), ptr(bias), 0.2, ptr(out), ptr(alpha), st,
                                      gnp)

            def aggregate_then_project():
                st = stream_handle(dev)
                check(LIB.vg_gemm(ptr(w_att), cin, ptr(x), cin, 1, None, 0, None, 0, ptr(sd), n, 2, n, cin, st),
                      "vg_gemm")
                ops.aggregate_fwd_raw(csr, cin, ptr(x), ptr(sd[0]), ptr(sd[1]), ptr(zero_b), 0.2, ptr(z), ptr(alpha),
                                      st)
                check(LIB.vg_gemm(ptr(z), cin, ptr(w), cin, 1, ptr(bias), 0, None, 0, ptr(out), cout, n, cout, cin,
                                  st), "vg_gemm")

            project_then_aggregate()
            ref = out.clone()
            aggregate_then_project()
            torch.cuda.synchronize()
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            rec = {"copies": copies, "rows": n, "edges": csr.num_edges, "cin": cin, "cout": cout,
                   "project_then_aggregate_us": round(timed(project_then_aggregate), 2),
                   "aggregate_then_project_us": round(timed(aggregate_then_project), 2),
                   "max_rel_diff": float(f"{err:.2e}")}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
