#!/bin/bash
# round 6: split Sinkhorn exchange without the acquire fence (sc1 slot loads) -- tests, then per-launch
# timing over the sibling count (FPM_SK_SPLIT) with / without the fence (FPM_SK_XACQ)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -k "stream or n512 or c5 or max_box or fp32_chain or block_order" -v --timeout 250 --timeout-method thread > gpurun_out/r06_noacq_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_noacq_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_noacq_tests.log
for b in 64 128; do for g in 2 4 8; do for x in 0 1; do
  FPM_SK_SPLIT=$g FPM_SK_XACQ=$x timeout -k 10 100 python tools/sk_stream_bench.py $b 512 20 t | sed "s/^/split=$g xacq=$x /" || exit 1
done; done; done
