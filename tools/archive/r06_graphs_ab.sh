#!/bin/bash
# round 6: whole-forward HIP graphs (FPM_GRAPHS) on the 128-pair forward and C3
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {  # tag batch env...
  local tag=$1 b=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 3 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --parity-pairs 0 > gpurun_out/r06_gr_$tag.json 2> gpurun_out/r06_gr_$tag.err || { tail -5 gpurun_out/r06_gr_$tag.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_gr_$tag.json'));print('$tag', '$*', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'selfcheck', d.get('timed_batch_selfcheck'))"
}
for rep in 1 2; do
  run s0_$rep 128 FPM_GRAPHS=0 || exit 1
  run s1_$rep 128 FPM_GRAPHS=1 || exit 1
  run c0_$rep 1024 FPM_GRAPHS=0 || exit 1
  run c1_$rep 1024 FPM_GRAPHS=1 || exit 1
done
