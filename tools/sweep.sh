#!/bin/bash
# bench under several (streams:chunks:tail) settings: bash tools/sweep.sh "2:8:0 2:8:1 2:8:2"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in $1; do
  IFS=: read s c t <<< "$cfg"
  FPM_TAIL=$t FPM_STREAMS=$s FPM_CHUNKS=$c timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/sw.json 2> gpurun_out/sw.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sw.json')); print('cfg $cfg', round(d['value'],1), 'pairs/s', round(d['ms_per_step'],2), 'ms', 'gpu-stage', round(1024e3/d['gpu_stage_pairs_per_s'],2), 'ms')"
done
