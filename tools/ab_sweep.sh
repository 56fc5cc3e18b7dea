#!/bin/bash
# A/B of library variants on the configs[4] inference sweep (bench.py's
# inference_sweep block), alternated twice: AB_VARIANTS="_x _y" bash tools/ab_sweep.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for v in "" ${AB_VARIANTS}; do
  L=$R/building-gan-graph-conditioned-architectural-volume-generation_amd/vgan/libvgan_hip$v.so
  VGAN_LIB=$L timeout -k 10 300 python bench.py --no-stress --no-cpu-baseline --no-fresh --no-bf16 --steps 5 \
    > $R/gpurun_out/abs_${v}_${rep}.json 2> /dev/null || exit 1
  python3 - "$v" "$rep" "$R/gpurun_out/abs_${v}_${rep}.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])["inference_sweep"]
print(f"v={sys.argv[1]} rep={sys.argv[2]} f16 {d['f16']['value']:.0f} samples/s ({d['f16']['ms_per_batch']:.4f} ms/batch)"
      f" f32 {d['f32']['value']:.0f} ({d['f32']['ms_per_batch']:.4f}); vg_hgat_fwd {d['roofline']['avg_launch_us']} us,"
      f" frac {d['roofline']['frac']}")
PY
done
done
