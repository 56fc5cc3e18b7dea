#!/bin/bash
# Library variant for an A/B (tools/ab_libs.sh, tools/ab_tn.sh):
#   tools/build_variant.sh <suffix> "<extra hipcc flags>" [sources...]
# recompiles the named sources (default: all) with the extra flags and links
# vgan/libvgan_hip<suffix>.so beside the default library (load it with VGAN_LIB).
set -euo pipefail
SUF=$1; FLAGS=$2; shift 2
D=$(cd "$(dirname "$0")/.." && pwd)/building-gan-graph-conditioned-architectural-volume-generation_amd/csrc
make -s -C "$D" > /dev/null
mkdir -p "$D/build_v$SUF"
OBJS=()
for o in "$D"/build/*.o; do
  b=$(basename "$o" .o)
  if [ "$b" != stamp ] && { [ $# -eq 0 ] || [[ " $* " == *" $b.hip "* ]]; }; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-pass-failed $FLAGS -c "$D/$b.hip" -o "$D/build_v$SUF/$b.o"
    OBJS+=("$D/build_v$SUF/$b.o")
  else
    OBJS+=("$o")
  fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "${OBJS[@]}" -o "$D/../vgan/libvgan_hip$SUF.so"
echo "built vgan/libvgan_hip$SUF.so"
