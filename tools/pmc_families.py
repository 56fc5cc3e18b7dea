"""Per-kernel-family HBM-side traffic and bandwidth of the training step.

usage: pmc_families.py PMC_DIR SUMMARY_TXT

PMC_DIR holds FETCH_SIZE.csv / WRITE_SIZE.csv of tools/pmc_step.sh (every
dispatch of a short bench.py run); SUMMARY_TXT is tools/profile_step.sh's
summary of the timed steps of the same build (tools/prof_summary.py: per
kernel total ms, count, average; "per step: N dispatches").  Traffic per
dispatch = (2 FETCH_SIZE + WRITE_SIZE) KiB (gfx950: FETCH_SIZE counts half of
a wide read; MI355X_MICROARCH.md), the bytes that left L2 (MALL hits
included: an upper bound on HBM bytes).  Prints a markdown table: family,
dispatches per step, average duration, average traffic, achieved GB/s and its
fraction of 8 TB/s, share of the timed kernel time.
"""
import csv
import re
import sys
from collections import defaultdict

PEAK = 8000.0  # GB/s


def family(name: str) -> str:
    m = re.search(r"::(k_\w+)", name)
    if m:
        return m.group(1)
    m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)", name)
    return "torch:" + m.group(1) if m else name[:40]


def traffic(path):
    per = defaultdict(float)
    fam = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[d] += float(r["Counter_Value"])
            fam[d] = family(r.get("Kernel_Name", ""))
    out = defaultdict(list)
    for d, v in per.items():
        out[fam[d]].append(v)
    return out


def main():
    pmc, summary = sys.argv[1], sys.argv[2]
    text = open(summary).read()
    m = re.search(r"per step: (\d+) dispatches, ([\d.]+) ms busy", text)
    per_step, busy_ms = int(m.group(1)), float(m.group(2))
    fetch = traffic(f"{pmc}/FETCH_SIZE.csv")
    write = traffic(f"{pmc}/WRITE_SIZE.csv")
    dur = defaultdict(lambda: [0, 0.0])
    for line in text.splitlines():
        r = re.match(r"^\s*([\d.]+) ms\s+(\d+) x\s+([\d.]+) us\s+(.*)$", line)
        if r:
            f = family(r.group(4))
            dur[f][0] += int(r.group(2))
            dur[f][1] += float(r.group(1))
    total = sum(v[1] for v in dur.values())
    steps = round(int(re.search(r"dispatches (\d+)\s+kernel-busy", text).group(1)) / per_step)
    print(f"Timed steps: {steps:.0f}; {per_step} dispatches and {busy_ms:.2f} ms of kernel time per step "
          f"(rocprofv3, serialised); families below cover {total / steps / busy_ms:.0%} of it.")
    print()
    print("| kernel family | dispatches / step | avg µs | avg traffic MB | GB/s | of 8 TB/s | share of kernel time |")
    print("|---|---|---|---|---|---|---|")
    for f, (n, ms) in sorted(dur.items(), key=lambda kv: -kv[1][1]):
        avg_us = ms * 1e3 / n
        if ms / steps / busy_ms < 0.005:
            continue
        fe, wr = fetch.get(f), write.get(f)
        if fe and wr:
            mb = (2 * sum(fe) / len(fe) + sum(wr) / len(wr)) * 1024 / 1e6
            gbs = mb * 1e6 / (avg_us * 1e3)
            cells = f"{mb:.2f} | {gbs:.0f} | {gbs / PEAK:.3f}"
        else:
            cells = "- | - | -"
        print(f"| `{f}` | {n / steps:.1f} | {avg_us:.2f} | {cells} | {ms / steps / busy_ms:.1%} |")


if __name__ == "__main__":
    main()
