#!/bin/bash
# A/B of environment knobs on one box: AB_ENVS="VAR=0 VAR=1" bash tools/ab_env.sh
# (several variables in one setting: comma-separated, "A=0,B=1")
# runs bench.py (no stress / CPU baseline) per setting, alternated twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for e in ${AB_ENVS}; do
  env ${e//,/ } timeout -k 10 120 python bench.py --no-stress --no-cpu-baseline --no-fresh --no-sweep --steps 30 > /dev/null 2> $R/gpurun_out/abenv_${rep}.err || exit 1
  echo "$e rep=$rep $(grep timed $R/gpurun_out/abenv_${rep}.err | sed 's/\[bench [0-9:]*\] //' | tr '\n' ' ')"
done
done
