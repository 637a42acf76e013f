#!/bin/bash
# round 6: 128-pair forward -- tail-group shape sweep (FPM_TAIL_GROUPS / FPM_TAIL_LAST / FPM_LSA_THREADS)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --batch 128 --steps 40 --warmup 5 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --parity-pairs 0 > gpurun_out/r06_ts_$tag.json 2> gpurun_out/r06_ts_$tag.err || { tail -5 gpurun_out/r06_ts_$tag.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_ts_$tag.json'));print('$tag', '$*', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d.get('host_lsa_ms_per_step',0),2))"
}
for rep in 1 2; do
  run base$rep FPM_TAIL_GROUPS=4 FPM_TAIL_LAST=0.5 || exit 1
  run l03_$rep FPM_TAIL_GROUPS=4 FPM_TAIL_LAST=0.3 || exit 1
  run g5_$rep FPM_TAIL_GROUPS=5 FPM_TAIL_LAST=0.4 || exit 1
  run g3_$rep FPM_TAIL_GROUPS=3 FPM_TAIL_LAST=0.4 || exit 1
  run t48_$rep FPM_TAIL_GROUPS=4 FPM_TAIL_LAST=0.5 FPM_LSA_THREADS=48 || exit 1
  run t16_$rep FPM_TAIL_GROUPS=4 FPM_TAIL_LAST=0.5 FPM_LSA_THREADS=16 || exit 1
done
