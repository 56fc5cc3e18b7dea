#!/bin/bash
# A/B: bench per library variant, alternated twice
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for v in "" ${AB_VARIANTS}; do
  L=$R/building-gan-graph-conditioned-architectural-volume-generation_amd/vgan/libvgan_hip$v.so
  VGAN_LIB=$L timeout -k 10 120 python bench.py --no-stress --no-cpu-baseline --no-fresh --no-sweep --steps 30 > /dev/null 2> $R/gpurun_out/ab_${v}_${rep}.err || exit 1
  echo "v=$v rep=$rep $(grep -E 'timed|aggregate_fwd|k_gemm16' $R/gpurun_out/ab_${v}_${rep}.err | tr '\n' ' ')"
done
done
