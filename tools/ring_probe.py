"""Where the wave-specialised ring aggregation (vg_gat_aggregate_fwd_ring)
waits: with a VG_RING_PROF=1 build (tools/build_variant.sh _ringprof
"-DVG_RING_PROF=1" gat_staged.hip, loaded with VGAN_LIB), every wave records
the clocks it spent in hand-over waits and its lifetime; printed per role
(loaders: waiting for a FREE slot, consumers: waiting for a FULL one) on the
configs[3] stress graph in lattice-block order, C = 128 and 64.

    VGAN_LIB=.../libvgan_hip_ringprof.so python tools/ring_probe.py

A VG_RING_PROF=2 build fills the same four counters with: consumers' waits
on the first slice ("softmax_frac") and on later slices ("gather_frac");
loaders' FREE -> loaded clocks ("softmax_frac") and item count ("gather_frac"
x life).
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

GNP = os.environ.get("RING_GNP", "0") == "1"  # RING_GNP=1: vg_gat_aggregate_fwd_ring_gnp


def main():
    from vgan import ops
    from vgan._lib import LIB, check, ptr, stream_handle
    from vgan.graph import GraphBatch
    from vgan.locality import blocked
    from vgan.synth import make_stress_building

    dev = torch.device("cuda", 0)
    vox = GraphBatch.from_data_list([blocked(make_stress_building(777, i)[1])[0] for i in range(8)]).to(dev)
    csr = ops.CSR(vox.edge_index, vox.num_nodes)
    n = csr.num_nodes
    rplan = csr.ring_plan()
    grid = 256
    for c in (128, 64):
        h = torch.randn(n, c, device=dev)
        a_s, a_d = 0.3 * torch.randn(n, device=dev), 0.3 * torch.randn(n, device=dev)
        bias = torch.randn(c, device=dev)
        out, alpha = torch.empty(n, c, device=dev), torch.empty(csr.num_edges, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)

        gnp = torch.empty(int(LIB.vg_gat_ring_gnp_floats(n, c)), device=dev) if GNP else None

        def run():
            if GNP:  # the _gnp form the drop-in dispatches (GraphNorm partials per 64-row tile)
                check(LIB.vg_gat_aggregate_fwd_ring_gnp(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(a_s),
                                                        ptr(a_d), ptr(bias), 0.2, ptr(out), ptr(alpha), ptr(rplan), n,
                                                        ptr(gnp), ptr(err), stream_handle(dev)), "ring_gnp")
                return
            check(LIB.vg_gat_aggregate_fwd_ring(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(a_s), ptr(a_d),
                                                ptr(bias), 0.2, ptr(out), ptr(alpha), ptr(rplan), ptr(err),
                                                stream_handle(dev)), "ring")

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        reps = []
        cold = torch.empty(512 * 1024 * 1024 // 4, device=dev) if os.environ.get("RING_COLD") == "1" else None
        for _ in range(int(os.environ.get("RING_REPS", "1"))):  # launches, each between events
            if cold is not None:  # RING_COLD=1: the 256 MB MALL flushed before each (bench.py's cold launches)
                cold.fill_(1.0)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            torch.cuda.synchronize()
            reps.append(round(a.elapsed_time(b) * 1e3, 1))
        rec = {"gnp": GNP, "C": c, "us": reps[-1], "us_reps": reps, "err": int(err.item())}
        if not hasattr(LIB._lib if hasattr(LIB, "_lib") else LIB, "vg_ring_prof_read"):
            print(json.dumps(rec), flush=True)  # a production build: times only
            continue
        buf = (ctypes.c_ulonglong * (grid * 16 * 4))()
        rec["rc"] = LIB.vg_ring_prof_read(buf, grid * 16 * 4)
        vals = list(buf)
        for role, waves in (("loader", range(0, int(os.environ.get("RING_LW", "4")))), ("consumer", range(int(os.environ.get("RING_LW", "4")), 16))):
            w = [vals[(g * 16 + v) * 4] for g in range(grid) for v in waves]
            t = [vals[(g * 16 + v) * 4 + 1] for g in range(grid) for v in waves]
            sm = [vals[(g * 16 + v) * 4 + 2] for g in range(grid) for v in waves]
            ga = [vals[(g * 16 + v) * 4 + 3] for g in range(grid) for v in waves]
            rec[role] = {"wait_clk_avg": round(sum(w) / len(w)), "life_clk_avg": round(sum(t) / len(t)),
                         "wait_frac": round(sum(w) / max(1, sum(t)), 3), "life_clk_max": max(t),
                         "softmax_frac": round(sum(sm) / max(1, sum(t)), 3),
                         "gather_frac": round(sum(ga) / max(1, sum(t)), 3)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
