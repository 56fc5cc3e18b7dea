set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for args in "--no-sweep --steps 20" "--no-sweep --steps 30" "--steps 20"; do
  timeout -k 10 200 python bench.py --no-stress --no-cpu-baseline --no-bf16 $args > /dev/null 2> $R/gpurun_out/fab.err || exit 1
  echo "$args rep=$rep: $(grep -E 'timed \(|fresh batches|sweep f' $R/gpurun_out/fab.err | sed 's/\[bench [0-9:]*\] //' | tr '\n' ' ')"
done
done
