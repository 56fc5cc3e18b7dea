set -o pipefail
R=$GRAFT_REPO_ROOT
for v in "" _p1 _p2; do
  VGAN_LIB=$R/building-gan-graph-conditioned-architectural-volume-generation_amd/vgan/libvgan_hip$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-bf16 > /dev/null 2> $R/gpurun_out/probe_lds$v.err || exit 1
  echo "v=$v $(grep 'stress C=' $R/gpurun_out/probe_lds$v.err | sed 's/\[bench [0-9:]*\] //' | tr '\n' ' ')"
done
