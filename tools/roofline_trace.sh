#!/bin/bash
# usage: tools/roofline_trace.sh <tag>
# rocprofv3 kernel trace + stats of `bench.py --roofline-only` (the step's mix
# of vg_gat_aggregate_fwd launches, graph-replayed -- the same replays the
# bench line's `roofline.avg_launch_us` is timed over with HIP events).
# Leaves gpurun_out/rooftrace_<tag>/{bench.json, kernel_stats.csv, summary.txt};
# summary.txt holds the average duration over every aggregate launch.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rooftrace_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
rm -rf "/tmp/rooftrace_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "/tmp/rooftrace_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --roofline-only --steps 20 "$@" > "$OUT/bench.json" 2> "$OUT/bench.log" || exit $?
T=$(find "/tmp/rooftrace_$TAG" -name "*kernel_trace.csv" | head -1)
S=$(find "/tmp/rooftrace_$TAG" -name "*kernel_stats.csv" | head -1)
[ -n "$S" ] && cp "$S" "$OUT/kernel_stats.csv"
[ -n "$T" ] || { echo "no kernel_trace.csv"; exit 1; }
python3 - "$T" "$OUT/bench.json" > "$OUT/summary.txt" <<'EOF'
import csv, json, re, sys
from collections import defaultdict
rows = [r for r in csv.DictReader(open(sys.argv[1])) if re.search(r"k_gat_fwd_(cp|ep)", r["Kernel_Name"])]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
by = defaultdict(list)
for r, x in zip(rows, d):
    by[re.search(r"(k_gat_fwd_\w+<[^>]*>)", r["Kernel_Name"]).group(1)].append(x)
bench = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"aggregate launches traced: {len(d)}; average duration {sum(d) / len(d):.3f} us "
      f"(rocprofv3 kernel trace, all replays incl. warm-up)")
print(f"bench.py --roofline-only (HIP events over the same replays): {bench}")
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k:32s} {len(v):6d} x {sum(v) / len(v):8.3f} us")
EOF
