#!/bin/bash
# round 6: pipeline chunks per 1024-pair forward (FPM_CHUNKS 4 / 6 / 8) at C3
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in 8 4 6 8 4 6; do
  FPM_CHUNKS=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --parity-pairs 0 > gpurun_out/r06_ch_$v.json 2> gpurun_out/r06_ch_$v.err || { tail -5 gpurun_out/r06_ch_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_ch_$v.json'));print('chunks=$v', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'lsa', round(d['host_lsa_ms_per_step'],1))"
done
