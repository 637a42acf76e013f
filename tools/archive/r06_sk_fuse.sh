#!/bin/bash
# round 6: fused row + column pass in the streaming Sinkhorn (FPM_SK_FUSE) -- tests, timing, C5 A/B
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -k "stream or n512 or c5 or max_box or fp32_chain or block_order or univ" -v --timeout 250 --timeout-method thread > gpurun_out/r06_fuse_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_fuse_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_fuse_tests.log
for b in 64 128; do for t in n t; do for f in 0 1; do
  FPM_SK_FUSE=$f timeout -k 10 100 python tools/sk_stream_bench.py $b 512 20 $t | sed "s/^/fuse=$f /" || exit 1
done; done; done
for f in 0 1 0 1; do
  FPM_SK_FUSE=$f timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-selfcheck > gpurun_out/r06_c5_fuse$f.json 2> gpurun_out/r06_c5_fuse$f.err || { tail -5 gpurun_out/r06_c5_fuse$f.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_c5_fuse$f.json'));print('c5 fuse=$f', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']))"
done
