#!/bin/bash
# A/B of environment knobs on the fresh-batch leg (plus the graphed step):
# AB_ENVS="VGAN_GEN=engine VGAN_GEN=autograd" bash tools/ab_fresh.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for e in ${AB_ENVS}; do
  env $e timeout -k 10 180 python bench.py --no-stress --no-cpu-baseline --no-sweep --no-bf16 --steps 30 > /dev/null 2> $R/gpurun_out/abfresh_${rep}.err || exit 1
  echo "$e rep=$rep $(grep -E 'timed|fresh' $R/gpurun_out/abfresh_${rep}.err | sed 's/\[bench [0-9:]*\] //' | tr '\n' ' ')"
done
done
