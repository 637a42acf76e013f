#!/bin/bash
# round 6: Hungarian pool size (FPM_LSA_THREADS 32 = 2x the 16-CPU share, 48, 64): 128-pair share line and C3
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {  # tag batch env...
  local tag=$1 b=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 3 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --parity-pairs 0 > gpurun_out/r06_lt_$tag.json 2> gpurun_out/r06_lt_$tag.err || { tail -5 gpurun_out/r06_lt_$tag.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_lt_$tag.json'));print('$tag', '$*', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d.get('host_lsa_ms_per_step',0),2))"
}
for rep in 1 2; do
  for t in 32 48 64; do run s${t}_$rep 128 FPM_LSA_THREADS=$t || exit 1; done
  for t in 32 48 64; do run c${t}_$rep 1024 FPM_LSA_THREADS=$t || exit 1; done
done
