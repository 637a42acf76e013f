#!/bin/bash
# GPU tests, then the default bench alternating an env switch: VAR=FPM_GNN_PACKED bash tools/ab.sh [a] [b]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=${VAR:-FPM_GEMM_PHASE}; A=${1:-1}; Bv=${2:-0}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
for z in $A $Bv $A $Bv; do
  env $V=$z timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ab$z.json 2> gpurun_out/ab$z.err || { tail gpurun_out/ab$z.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab$z.json')); r=d['roofline']
print('$V=$z', round(d['value']), 'gpu-stage', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d['host_lsa_ms_per_step'],1), 'gemm', round(r['achieved']), round(r['isolated_achieved']))"
done
