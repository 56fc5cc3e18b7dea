"""configs[3] stress graph: the register gather, the persistent staged kernel
(vg_gat_aggregate_fwd_staged) and the wave-specialised ring kernel
(vg_gat_aggregate_fwd_ring) in three voxel numberings, cold MALL, HIP events.
One JSON line per (order, kernel, C).

    python tools/staged_probe.py [--reps 20] [--orders rowmajor,tiled,blocked,morton]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vgan import ops  # noqa: E402
from vgan._lib import LIB, check, ptr, stream_handle  # noqa: E402
from vgan.graph import GraphBatch  # noqa: E402
from vgan.locality import blocked, tiled  # noqa: E402
from vgan.synth import make_stress_building  # noqa: E402


def agg_bytes(n, e, c):
    return 4 * (2 * n * c + 2 * n + e + (n + 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--orders", default="rowmajor,tiled,blocked")
    ap.add_argument("--channels", default="128,64")
    ap.add_argument("--buildings", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    items = [make_stress_building(777, i)[1] for i in range(args.buildings)]
    scratch = torch.empty(512 * 1024 * 1024 // 4, device=dev)
    st = stream_handle(dev)
    for order in args.orders.split(","):
        vs = (items if order == "rowmajor" else [tiled(v, 4)[0] for v in items] if order == "tiled"
              else [blocked(v, blocks="morton" if order == "morton" else "rowmajor")[0] for v in items])
        vox = GraphBatch.from_data_list(vs).to(dev)
        csr = ops.CSR(vox.edge_index, vox.num_nodes)
        n, e = csr.num_nodes, csr.num_edges
        plan = csr.stage_plan()
        rplan = csr.ring_plan()
        tiles = csr.stage_tiles()
        uc = plan[:tiles]
        info = {"order": order, "nodes": n, "edges": e, "staged_tiles": int((uc > 0).sum()),
                "global_tiles": int((uc < 0).sum()),
                "distinct_per_64_tile": round(float(uc.clamp_min(0).sum()) / max(1, int((uc > 0).sum())), 1)}
        print(json.dumps(info), flush=True)
        for c in [int(x) for x in args.channels.split(",")]:
            torch.manual_seed(c)
            h = torch.randn(n, c, device=dev)
            a_s, a_d = 0.3 * torch.randn(n, device=dev), 0.3 * torch.randn(n, device=dev)
            bias = torch.randn(c, device=dev)
            out, alpha = torch.empty(n, c, device=dev), torch.empty(e, device=dev)
            out2, alpha2 = torch.empty(n, c, device=dev), torch.empty(e, device=dev)
            out3, alpha3 = torch.empty(n, c, device=dev), torch.empty(e, device=dev)
            err = torch.zeros(1, dtype=torch.int32, device=dev)

            def reg():
                ops.aggregate_fwd_raw(csr, c, ptr(h), ptr(a_s), ptr(a_d), ptr(bias), 0.2, ptr(out), ptr(alpha), st)

            def staged():
                check(LIB.vg_gat_aggregate_fwd_staged(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(a_s),
                                                      ptr(a_d), ptr(bias), 0.2, ptr(out2), ptr(alpha2), ptr(plan), st),
                      "staged")

            def ring():
                check(LIB.vg_gat_aggregate_fwd_ring(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(a_s), ptr(a_d),
                                                    ptr(bias), 0.2, ptr(out3), ptr(alpha3), ptr(rplan), ptr(err), st),
                      "ring")

            def timed(fn, cold=True):
                for _ in range(3):
                    fn()
                ts = []
                for _ in range(args.reps):
                    if cold:
                        scratch.fill_(1.0)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    fn()
                    b.record()
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b) * 1e3)
                ts.sort()
                return sum(ts) / len(ts), ts[len(ts) // 2]

            by = agg_bytes(n, e, c)
            for name, fn in (("register", reg), ("staged", staged), ("ring", ring)):
                avg, med = timed(fn)
                warm, _ = timed(fn, cold=False)
                print(json.dumps({"order": order, "kernel": name, "C": c, "avg_us": round(avg, 2),
                                  "median_us": round(med, 2), "warm_us": round(warm, 2),
                                  "frac": round(by / (avg * 1e-6) / 8e12, 4)}), flush=True)
            torch.cuda.synchronize()
            if int(err.item()) != 0:
                raise RuntimeError("ring: a hand-over wait expired")
            same = all(torch.equal(out, o) and torch.equal(alpha, a) for o, a in ((out2, alpha2), (out3, alpha3)))
            print(json.dumps({"order": order, "C": c, "bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
