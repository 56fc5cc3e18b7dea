"""Split a rocprofv3 kernel trace of `phase_times.py --gaps` into its last
three gap-separated segments (labels, critic, gen) and print, per phase, the
dispatch count, summed kernel time and the kernels by family.

usage: phase_kernels.py TRACE.csv
"""
import csv
import re
import sys
from collections import defaultdict


def family(name: str) -> str:
    m = re.search(r"::(k_\w+)", name)
    if m:
        return m.group(1)
    m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)", name)
    if m:
        f = re.search(r"at::native::(?:\(anonymous namespace\)::)?\w+<[^,]*, at::native::(?:\(anonymous namespace\)::)?(\w+)", name)
        return "torch:" + m.group(1) + (":" + f.group(1) if f else "")
    return name[:40]


def main():
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(sys.argv[1])))
    cuts = [i + 1 for i in range(len(rows) - 1) if rows[i + 1][0] - rows[i][1] > 50_000_000]
    segs = [rows[a:b] for a, b in zip([0] + cuts, cuts + [len(rows)])][-3:]
    for name, seg in zip(("labels", "critic", "gen"), segs):
        fam = defaultdict(lambda: [0, 0.0])
        for s, e, k in seg:
            f = fam[family(k)]
            f[0] += 1
            f[1] += (e - s) / 1e3
        busy = sum(v[1] for v in fam.values())
        span = (seg[-1][1] - seg[0][0]) / 1e3
        print(f"== {name}: {len(seg)} dispatches, busy {busy:.1f} us, span {span:.1f} us")
        for k, (n, us) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
            print(f"   {us:8.1f} us {n:5d} x {us / n:6.2f}  {k}")


if __name__ == "__main__":
    main()
