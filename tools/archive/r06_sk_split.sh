#!/bin/bash
# round 6: split streaming Sinkhorn (FPM_SK_SPLIT workgroups per pair) -- parity tests, per-launch
# timing (split 1 vs 4, both layouts, 20 steps, 64 and 128 pairs), C5 bench A/B
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "stream or n512 or c5 or sinkhorn" -v --timeout 200 --timeout-method thread > gpurun_out/r06_split_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_split_tests.log | tail -20; exit 1; }
grep -cE "PASSED" gpurun_out/r06_split_tests.log
for g in 1 2; do for b in 64 128; do for t in n t; do
  FPM_SK_SPLIT=$g timeout -k 10 120 python tools/sk_stream_bench.py $b 512 20 $t | sed "s/^/split=$g /" || exit 1
done; done; done
for g in ${GS:-1 2 4 1 2 4}; do
  FPM_SK_SPLIT=$g timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-selfcheck > gpurun_out/r06_c5_split$g.json 2> gpurun_out/r06_c5_split$g.err || { tail -5 gpurun_out/r06_c5_split$g.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_c5_split$g.json'));print('split=$g', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'gate', (d.get('parity_gate') or {}).get('passed'))"
done
