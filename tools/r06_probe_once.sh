#!/bin/bash
# round 6: C4 probe SplineConv once per forward (prologue) -- bit identity + C4 parity tests, C4 bench
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -k "probe or c4 or gallery or shard" -v --timeout 250 --timeout-method thread > gpurun_out/r06_probe_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_probe_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_probe_tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r06_c4_probe$r.json 2> gpurun_out/r06_c4_probe$r.err || { tail -5 gpurun_out/r06_c4_probe$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_c4_probe$r.json'));print('c4', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'selfcheck', d.get('timed_batch_selfcheck'))"
done
