#!/bin/bash
# usage: tools/profile_step.sh <tag> <steps> [extra bench args...]
# rocprofv3 kernel trace of `bench.py --profile`; leaves gpurun_out/prof_<tag>/
# {summary.txt (timed steps only), kernel_stats.csv, bench.json, bench.log}
set -o pipefail
TAG=$1; STEPS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --profile --steps $STEPS "$@" > $OUT/bench.json 2> $OUT/bench.log
rc=$?
T=$(find /tmp/prof_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$T" ] && python3 $R/tools/prof_summary.py $T ${TOP:-45} --after-gap --gaps --steps $STEPS ${SEQ:+--seq $SEQ} ${DUMP:+--dump-step} > $OUT/summary.txt
S=$(find /tmp/prof_$TAG -name "*kernel_stats.csv" | head -1)
[ -n "$S" ] && cp $S $OUT/kernel_stats.csv
exit $rc
