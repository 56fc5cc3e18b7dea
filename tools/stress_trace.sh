#!/bin/bash
# usage: tools/stress_trace.sh <tag>
# rocprofv3 kernel trace + stats of `bench.py --stress-only`: the configs[3]
# ring aggregations (8 x 50k stress buildings, lattice-block numbering,
# C = 128, a 512 MB scratch fill before every launch -- the bench's cold-MALL
# roofline_stress launches), plain and with the GraphNorm partials.
# Leaves gpurun_out/stresstrace_<tag>/{bench.json, kernel_stats.csv,
# summary.txt}; summary.txt's first line is the mean duration of the plain
# ring kernel (bench.py prices roofline_stress on it), then per variant.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stresstrace_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
rm -rf "/tmp/stresstrace_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "/tmp/stresstrace_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --stress-only "$@" > "$OUT/bench.json" 2> "$OUT/bench.log" || exit $?
T=$(find "/tmp/stresstrace_$TAG" -name "*kernel_trace.csv" | head -1)
S=$(find "/tmp/stresstrace_$TAG" -name "*kernel_stats.csv" | head -1)
[ -n "$S" ] && cp "$S" "$OUT/kernel_stats.csv"
[ -n "$T" ] || { echo "no kernel_trace.csv"; exit 1; }
python3 - "$T" "$OUT/bench.json" > "$OUT/summary.txt" <<'PY'
import csv, json, re, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_gat_fwd_ring" in r["Kernel_Name"]]
by = {}
for r in rows:
    gnp = bool(re.search(r"Lb1E|, true>", r["Kernel_Name"]))
    by.setdefault(gnp, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
plain = by.get(False, [])
bench = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"ring launches traced: {len(plain)}; average duration {sum(plain) / max(1, len(plain)):.3f} us "
      f"(rocprofv3 kernel trace, k_gat_fwd_ring plain, C=128, cold MALL, incl. 3 warm-up launches)")
g = by.get(True, [])
print(f"ring_gnp launches traced: {len(g)}; average duration {sum(g) / max(1, len(g)):.3f} us")
print(f"bench.py --stress-only (HIP events over the same launches): {bench}")
PY
cat "$OUT/summary.txt"
