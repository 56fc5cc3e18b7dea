# A/B of the grouped weight-gradient launch: tools/tn_probe.py under each
# library variant (the default library and AB_VARIANTS, suffixes of vgan/libvgan_hip<suffix>.so), twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for round in 1 2; do
  for v in "" ${AB_VARIANTS}; do
    VGAN_LIB=$R/building-gan-graph-conditioned-architectural-volume-generation_amd/vgan/libvgan_hip$v.so \
      timeout -k 10 200 python tools/tn_probe.py --reps 50 > $R/gpurun_out/tn_probe$v.json 2> $R/gpurun_out/tn_probe$v.err || exit 1
    echo "round $round v=$v"; python3 -c "
import json,sys
for l in open('$R/gpurun_out/tn_probe$v.json'):
    d=json.loads(l); print(' list', d['list'], d['products'], 'prods', d['us'], 'us', d['GBs'], 'GB/s', d['TFLOPs'], 'TF')"
  done
done
