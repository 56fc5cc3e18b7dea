"""Summarise a rocprofv3 --kernel-trace CSV (kernel busy time vs wall span,
top kernels) so the multi-MB trace itself need not be kept.

usage: prof_summary.py TRACE.csv [TOP] [--after-gap] [--steps K]
  --after-gap  keep only the kernels after the LAST idle gap of >= 40 ms
               (bench.py --profile sleeps 50 ms before its timed steps and
               returns right after them; staging and capture gaps come earlier)
  --steps K    also report per-step dispatch counts / busy time
  --gaps       also report the idle gaps between consecutive dispatches of
               the kept region: total per size bucket and the largest ones
               with the kernels on either side
  --seq PAT    per-launch durations, in order, of the kernels whose name
               contains PAT (the first step's)
"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
path = args[0]
top = int(args[1]) if len(args) > 1 else 40
after_gap = "--after-gap" in sys.argv
steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 0
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
rows.sort()
if after_gap and len(rows) > 1:
    gaps = [(rows[i + 1][0] - rows[i][1], i) for i in range(len(rows) - 1)]
    long_gaps = [gi for gi in gaps if gi[0] >= 40_000_000]
    g, i = long_gaps[-1] if long_gaps else max(gaps)
    print(f"last idle gap >= 40 ms: {g / 1e6:.1f} ms after dispatch {i}; keeping the {len(rows) - i - 1} "
          f"dispatches after it")
    rows = rows[i + 1:]
tot = defaultdict(lambda: [0, 0.0])
busy = 0.0
for s, e, name in rows:
    tot[name][0] += 1
    tot[name][1] += (e - s) / 1e3
    busy += (e - s) / 1e3
t0, t1 = rows[0][0], max(e for _, e, _ in rows)
print(f"dispatches {len(rows)}  kernel-busy {busy / 1e3:.2f} ms  span {(t1 - t0) / 1e6:.2f} ms")
if steps:
    print(f"per step: {len(rows) / steps:.0f} dispatches, {busy / 1e3 / steps:.3f} ms busy, "
          f"{(t1 - t0) / 1e6 / steps:.3f} ms span")
if "--gaps" in sys.argv:
    import re

    def short(n):
        m = re.search(r"::(k_\w+)", n)
        return m.group(1) if m else n[:40]

    buckets = [(1, "<1 us"), (5, "1-5 us"), (20, "5-20 us"), (100, "20-100 us"), (float("inf"), ">=100 us")]
    acc = {b: [0, 0.0] for _, b in buckets}
    big = []
    end = rows[0][1]
    for i in range(1, len(rows)):
        g = (rows[i][0] - end) / 1e3
        end = max(end, rows[i][1])
        if g <= 0:
            continue
        for lim, b in buckets:
            if g < lim:
                acc[b][0] += 1
                acc[b][1] += g
                break
        big.append((g, short(rows[i - 1][2]), short(rows[i][2])))
    div = steps or 1
    print("idle gaps per step: " + ", ".join(f"{b}: {acc[b][0] / div:.0f} x, {acc[b][1] / div:.1f} us"
                                              for _, b in buckets))
    for g, a, b in sorted(big, reverse=True)[:12]:
        print(f"  gap {g:8.1f} us  {a} -> {b}")
if "--dump-step" in sys.argv and steps:  # the first timed step's kernels in order, runs of one name folded
    import re

    per = len(rows) // steps
    out, prev, cnt, t = [], None, 0, 0.0
    for s_, e_, name in rows[:per] + [(0, 0, None)]:
        m = re.search(r"::(k_\w+)", name) if name else None
        short = (m.group(1) if m else name[:60]) if name else None
        if short == prev:
            cnt += 1
            t += (e_ - s_) / 1e3
            continue
        if prev is not None:
            out.append(f"{prev} x{cnt} {t:.1f}us" if cnt > 1 else f"{prev} {t:.1f}us")
        prev, cnt, t = short, 1, (e_ - s_) / 1e3
    print("first step, in order:")
    for line in out:
        print("   ", line)
if "--seq" in sys.argv:  # per-launch durations (in order) of kernels whose name contains the pattern
    pat = sys.argv[sys.argv.index("--seq") + 1]
    seq = [(e - s) / 1e3 for s, e, name in rows if pat in name]
    per = len(seq) // steps if steps else len(seq)
    print(f"{pat}: {len(seq)} launches; first step: " + " ".join(f"{v:.1f}" for v in seq[:per]))
for name, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{us / 1e3:9.3f} ms {n:7d} x {us / n:8.2f} us  {name[:110]}")
