# usage: tools/pmc_kernel.sh <tag> <kernel-regex> "<counters>" <cmd...>
# one rocprofv3 --pmc pass (counters only, no trace domains) restricted to one
# kernel; leaves gpurun_out/pmc_<tag>/counters.csv + a per-counter mean summary
set -o pipefail
TAG=$1; RE=$2; CTRS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && rm -rf /tmp/pmc_$TAG
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-include-regex "$RE" -d /tmp/pmc_$TAG -o run --output-format csv -- "$@" > $OUT/run.log 2>&1
rc=$?
C=$(find /tmp/pmc_$TAG -name "*counter_collection.csv" | head -1)
[ -n "$C" ] && cp $C $OUT/counters.csv && python3 - "$C" > $OUT/summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    acc[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:60s} {c:28s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
PY
cat $OUT/summary.txt 2>/dev/null
exit $rc
