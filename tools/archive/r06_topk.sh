#!/bin/bash
# round 6: soft top-k continuation test without a pass -- parity tests, then per-launch timing
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_ops.py tests/test_train.py -m gpu -k "topk or soft or gated or forward" -v --timeout 200 --timeout-method thread > gpurun_out/r06_topk_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_topk_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_topk_tests.log
B=32 timeout -k 10 120 python tools/topk_steps.py && B=128 timeout -k 10 120 python tools/topk_steps.py
