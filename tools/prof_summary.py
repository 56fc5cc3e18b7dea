"""Summarise a rocprofv3 --kernel-trace CSV (kernel busy time vs wall span,
top kernels) so the multi-MB trace itself need not be kept."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
tot = defaultdict(lambda: [0, 0.0])
t0, t1, busy = None, None, 0.0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    tot[name][0] += 1
    tot[name][1] += (e - s) / 1e3
    busy += (e - s) / 1e3
    t0 = s if t0 is None else min(t0, s)
    t1 = e if t1 is None else max(t1, e)
print(f"dispatches {len(rows)}  kernel-busy {busy / 1e3:.2f} ms  span {(t1 - t0) / 1e6:.2f} ms")
for name, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f"{us / 1e3:9.3f} ms {n:7d} x {us / n:8.2f} us  {name[:110]}")
