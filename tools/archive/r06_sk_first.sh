#!/bin/bash
# round 6: streaming Sinkhorn vectorised first step -- parity tests, per-launch timing (2 and 20 steps, both
# layouts) for FPM_SK_STREAM_RW 1 (old scalar path) and 4, then the C5 bench
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "stream or n512 or c5 or sinkhorn" -v --timeout 200 --timeout-method thread > gpurun_out/r06_sk_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_sk_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_sk_tests.log
for rw in 1 4; do for it in 2 20; do for t in n t; do
  FPM_SK_STREAM_RW=$rw timeout -k 10 120 python tools/sk_stream_bench.py 128 512 $it $t || exit 1
done; done; done
for rw in 1 4; do
  FPM_SK_STREAM_RW=$rw timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-selfcheck > gpurun_out/r06_c5_rw$rw.json 2> gpurun_out/r06_c5_rw$rw.err || { tail -5 gpurun_out/r06_c5_rw$rw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_c5_rw$rw.json'));print('rw=$rw', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'gate', (d.get('parity_gate') or {}).get('passed'))"
done
