#!/bin/bash
# round 6: streaming Sinkhorn row step (multi-row + DPP) -- tests, then C5 A/B (FPM_SK_STREAM_RW 1 vs 4)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "stream or n512 or c5" -v --timeout 200 --timeout-method thread > gpurun_out/r06_c5_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_c5_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_c5_tests.log
for rw in ${RWS:-1 4 1 4}; do
  FPM_SK_STREAM_RW=$rw timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-selfcheck > gpurun_out/r06_c5_rw$rw.json 2> gpurun_out/r06_c5_rw$rw.err || { tail -5 gpurun_out/r06_c5_rw$rw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_c5_rw$rw.json'));print('rw=$rw', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'gate', (d.get('parity_gate') or {}).get('passed'))"
done
