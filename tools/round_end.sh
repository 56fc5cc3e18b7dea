#!/bin/bash
# The round's GPU records in one call: usage tools/round_end.sh <tag>
#   full `pytest -m gpu`, smoke(), the default bench line, the scatter-kernel
#   roofline trace and PMC passes, and a kernel trace of the timed step.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final_$TAG
mkdir -p "$O"
cd "$R" || exit 1
echo "[round_end] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.txt" 2>&1 || exit $?
tail -1 "$O/pytest_gpu.txt"
echo "[round_end] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || exit $?
echo "[round_end] bench"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.log" || exit $?
cat "$O/bench.json"
echo "[round_end] roofline trace"
bash tools/roofline_trace.sh "$TAG" --gnp || exit $?
echo "[round_end] pmc"
bash tools/pmc_roofline.sh "${TAG}_gnp" --gnp || exit $?
echo "[round_end] step trace"
cd "$R" && bash tools/profile_step.sh "$TAG" 10 || exit $?
echo "[round_end] done"
