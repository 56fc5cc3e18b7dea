#!/bin/bash
# usage: tools/profile_fresh.sh <tag> <steps> <variant>
# rocprofv3 kernel trace of tools/fresh_probe.py (one variant): device busy
# time, idle gaps and dispatches per fresh-batch step; leaves
# gpurun_out/prof_<tag>/{summary.txt, probe.jsonl, probe.log}
set -o pipefail
TAG=$1; STEPS=$2; VAR=${3:-staged}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$TAG -o run --output-format csv -- python3 $R/tools/fresh_probe.py --steps $STEPS --variants $VAR > $OUT/probe.jsonl 2> $OUT/probe.log
rc=$?
T=$(find /tmp/prof_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$T" ] && python3 $R/tools/prof_summary.py $T ${TOP:-30} --after-gap --gaps --steps $STEPS > $OUT/summary.txt
exit $rc
