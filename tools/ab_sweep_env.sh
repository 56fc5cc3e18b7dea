#!/bin/bash
# A/B of environment settings on the configs[4] inference sweep (bench.py's
# inference_sweep block), alternated twice: AB_ENVS="VAR=1 VAR=2" bash tools/ab_sweep_env.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for e in ${AB_ENVS}; do
  env ${e//,/ } timeout -k 10 300 python bench.py --no-stress --no-cpu-baseline --no-fresh --no-bf16 --steps 5 \
    > $R/gpurun_out/abse_${rep}.json 2> /dev/null || exit 1
  python3 - "$e" "$rep" "$R/gpurun_out/abse_${rep}.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])["inference_sweep"]
print(f"{sys.argv[1]} rep={sys.argv[2]} f16 {d['f16']['value']:.0f} samples/s ({d['f16']['ms_per_batch']:.4f} ms/batch)"
      f" f32 {d['f32']['value']:.0f} ({d['f32']['ms_per_batch']:.4f})")
PY
done
done
