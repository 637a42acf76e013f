#!/bin/bash
# bench under several (streams, chunks) settings: bash tools/sweep.sh "2:8 3:8 2:4 4:16"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for sc in $1; do
  s=${sc%%:*}; c=${sc##*:}
  FPM_STREAMS=$s FPM_CHUNKS=$c timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/sw_$s_$c.json 2> gpurun_out/sw.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/sw_$s_$c.json')); print('streams=$s chunks=$c', round(d['value'],1), 'pairs/s', round(d['ms_per_step'],2), 'ms', 'gpu-stage', round(1024e3/d['gpu_stage_pairs_per_s'],2), 'ms')"
done
