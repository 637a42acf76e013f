#!/bin/bash
# round 6: 128-pair forward -- AFA-U over the whole chunk vs per tail group (FPM_TAIL_AFAU_ALL), share line
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in ${VS:-0 1 0 1}; do
  FPM_TAIL_AFAU_ALL=$v timeout -k 10 300 python bench.py --batch 128 --steps 40 --warmup 5 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --parity-pairs 0 > gpurun_out/r06_tail_$v.json 2> gpurun_out/r06_tail_$v.err || { tail -5 gpurun_out/r06_tail_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_tail_$v.json'));print('afau_all=$v', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'selfcheck', d.get('timed_batch_selfcheck'))"
done
