"""Summarise the PMC passes of tools/pmc_roofline.sh for the scatter kernel.

usage: pmc_summary.py DIR   (DIR holds FETCH_SIZE.csv, WRITE_SIZE.csv, bench_*.json)

Per dispatch of the aggregate kernels (k_gat_fwd_cp / k_gat_fwd_ep):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide (16 B/lane) coalesced read (MI355X_MICROARCH.md, HBM), so
  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024  bytes per launch.
Both counters are taken at the L2's memory side, so Infinity-Cache (MALL)
hits are included: the figure is "bytes that left L2", an upper bound on HBM
bytes.  Prints one JSON object (averages over all aggregate dispatches) next
to the algorithmic bytes per launch from the same run.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

KERNELS = ("k_gat_fwd_cp", "k_gat_fwd_ep")


def per_dispatch(path):
    vals = defaultdict(float)
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if not any(k in name for k in KERNELS):
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[d] += float(r["Counter_Value"])
            names[d] = name
    return vals, names


def main():
    d = sys.argv[1]
    fetch, names = per_dispatch(os.path.join(d, "FETCH_SIZE.csv"))
    write, _ = per_dispatch(os.path.join(d, "WRITE_SIZE.csv"))
    bench = {}
    try:
        with open(os.path.join(d, "bench_FETCH_SIZE.json")) as f:
            bench = json.loads(f.read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        pass
    nf, nw = len(fetch), len(write)
    avg_fetch_kib = sum(fetch.values()) / max(nf, 1)
    avg_write_kib = sum(write.values()) / max(nw, 1)
    traffic = (2.0 * avg_fetch_kib + avg_write_kib) * 1024.0
    by_kernel = defaultdict(list)
    for k, v in fetch.items():
        m = re.search(r"(k_gat_fwd_\w+<[^>]*>)", names[k])
        by_kernel[m.group(1) if m else names[k][:60]].append(v)
    out = {
        "kernel": "vg_gat_aggregate_fwd (k_gat_fwd_cp / k_gat_fwd_ep)",
        "dispatches_fetch": nf,
        "dispatches_write": nw,
        "avg_fetch_size_kib": round(avg_fetch_kib, 2),
        "avg_write_size_kib": round(avg_write_kib, 2),
        "traffic_bytes_per_launch": int(traffic),
        "algorithmic_bytes_per_launch": bench.get("avg_bytes"),
        "traffic_over_algorithmic": (round(traffic / bench["avg_bytes"], 3) if bench.get("avg_bytes") else None),
        "correction": "traffic = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950: FETCH_SIZE counts half of wide reads)",
        "avg_fetch_kib_by_kernel": {k: round(sum(v) / len(v), 2) for k, v in sorted(by_kernel.items())},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
