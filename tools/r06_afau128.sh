#!/bin/bash
# round 6: AFA-U fused instance norms for 128-keypoint boxes (two pairs per tile) -- kernel tests
# first, then the forwards, then the C4 A/B (each step stops the call on failure)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "norm_max_fused or norm_out_fused" -v --timeout 150 --timeout-method thread > gpurun_out/r06_afau128_k.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_afau128_k.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_afau128_k.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "fused_forward or gated or c4 or n128 or c2" -v --timeout 250 --timeout-method thread > gpurun_out/r06_afau128_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_afau128_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_afau128_tests.log
for v in 0 1 0 1; do
  FPM_AFAU_FUSE=$v timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --no-selfcheck > gpurun_out/r06_c4_fuse$v.json 2> gpurun_out/r06_c4_fuse$v.err || { tail -5 gpurun_out/r06_c4_fuse$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_c4_fuse$v.json'));print('c4 fuse=$v', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'gate', (d.get('parity_gate') or {}).get('passed'))"
done
