#!/bin/bash
# usage: tools/pmc_step.sh <tag>
# HBM-side traffic of every kernel of the training step: two rocprofv3 PMC
# passes (FETCH_SIZE, WRITE_SIZE; one counter per pass) over a short
# `bench.py` run.  Leaves gpurun_out/pmcstep_<tag>/{FETCH_SIZE,WRITE_SIZE}.csv;
# tools/pmc_families.py joins them with a kernel_stats.csv of the same build.
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcstep_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for CNT in FETCH_SIZE WRITE_SIZE; do
  rm -rf "/tmp/pmcs_$CNT"
  timeout -s KILL 300 rocprofv3 --pmc $CNT --output-format csv -d "/tmp/pmcs_$CNT" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-stress > "$OUT/bench_$CNT.json" 2> "$OUT/bench_$CNT.log" || exit $?
  F=$(find "/tmp/pmcs_$CNT" -name "*counter_collection.csv" | head -1)
  [ -n "$F" ] || { echo "no counter_collection.csv for $CNT"; exit 1; }
  cp "$F" "$OUT/$CNT.csv"
done
