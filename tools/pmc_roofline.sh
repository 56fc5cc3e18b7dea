#!/bin/bash
# usage: tools/pmc_roofline.sh <tag> [extra bench.py args, e.g. --gnp]
# HBM-side traffic of the scatter kernel (vg_gat_aggregate_fwd) from
# rocprofv3 PMC counters: one pass per counter (FETCH_SIZE and WRITE_SIZE do
# not fit one pass on gfx950), each over `bench.py --roofline-only` (the step's
# mix of aggregate launches, graph-replayed).  Leaves
# gpurun_out/pmc_<tag>/{FETCH_SIZE,WRITE_SIZE}.csv, bench_*.json and
# summary.json (tools/pmc_summary.py).
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for CNT in FETCH_SIZE WRITE_SIZE; do
  rm -rf "/tmp/pmc_$CNT"
  timeout -s KILL 240 rocprofv3 --pmc $CNT --output-format csv -d "/tmp/pmc_$CNT" -o run -- \
    python3 "$R/bench.py" --roofline-only --steps 5 "$@" > "$OUT/bench_$CNT.json" 2> "$OUT/bench_$CNT.log" || exit $?
  F=$(find "/tmp/pmc_$CNT" -name "*counter_collection.csv" | head -1)
  [ -n "$F" ] || { echo "no counter_collection.csv for $CNT"; exit 1; }
  cp "$F" "$OUT/$CNT.csv"
done
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json"
