#!/bin/bash
# round 4: bf16 scatter SplineConv backward without the unread fp32 cell rows -- training tests,
# then an interleaved training-step A/B (FPM_SCATTER_F32_ROWS=1: the old writes)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r04ae}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train.py -m gpu \
    > gpurun_out/${TAG}_train_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_train_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_train_tests.log
for cfg in "FPM_SCATTER_F32_ROWS=0" "FPM_SCATTER_F32_ROWS=1" "FPM_SCATTER_F32_ROWS=0" "FPM_SCATTER_F32_ROWS=1" "FPM_SCATTER_F32_ROWS=0" "FPM_SCATTER_F32_ROWS=1"; do
  env $cfg timeout -k 10 300 python tools/train_bench.py --cpu-pairs 0 >> gpurun_out/${TAG}_scatter_ab.txt 2>> gpurun_out/${TAG}_scatter_ab.err || { tail -30 gpurun_out/${TAG}_scatter_ab.err; exit 1; }
  echo "cfg=$cfg" >> gpurun_out/${TAG}_scatter_ab.txt
done
cat gpurun_out/${TAG}_scatter_ab.txt
