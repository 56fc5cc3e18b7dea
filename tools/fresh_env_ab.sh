#!/bin/bash
# A/B of environment settings on the fresh-batch leg: AB_ENVS="A=1 A=2" bash tools/fresh_env_ab.sh
# (several variables in one setting: comma-separated), alternated twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for e in ${AB_ENVS}; do
  env ${e//,/ } timeout -k 10 200 python bench.py --no-stress --no-cpu-baseline --no-sweep --no-bf16 --steps 30 > /dev/null 2> $R/gpurun_out/fenv.err || exit 1
  echo "$e rep=$rep: $(grep -E 'timed \(|fresh batches' $R/gpurun_out/fenv.err | sed 's/\[bench [0-9:]*\] //' | tr '\n' ' ')"
done
done
