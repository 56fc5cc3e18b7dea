#!/bin/bash
# usage: tools/sweep_trace.sh <tag>
# rocprofv3 kernel trace + stats of the configs[4] f16 sweep (tools/infer_sweep.py
# --graphs 1024, f16 only): per-kernel totals per batch forward.
# Leaves gpurun_out/sweeptrace_<tag>/{summary.txt, kernel_stats.csv, run.json}
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sweeptrace_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
rm -rf "/tmp/sweeptrace_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "/tmp/sweeptrace_$TAG" -o run --output-format csv -- \
  python3 "$R/tools/infer_sweep.py" --graphs 1024 --dtype f16 > "$OUT/run.json" 2> "$OUT/run.log" || exit $?
S=$(find "/tmp/sweeptrace_$TAG" -name "*kernel_stats.csv" | head -1)
T=$(find "/tmp/sweeptrace_$TAG" -name "*kernel_trace.csv" | head -1)
[ -n "$S" ] && cp "$S" "$OUT/kernel_stats.csv"
[ -n "$T" ] && python3 "$R/tools/prof_summary.py" "$T" 40 > "$OUT/summary.txt"
head -45 "$OUT/summary.txt"
