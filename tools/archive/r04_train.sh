#!/bin/bash
# round 4: training tests, then the training-step bench (+ kernel stats) and the torch-op probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r04f}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train.py \
    > gpurun_out/${TAG}_train_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_train_tests.log; exit 1; }
bash tools/gpu_train.sh > gpurun_out/${TAG}_train.txt 2>&1 || { tail -30 gpurun_out/${TAG}_train.txt; exit 1; }
timeout -k 10 300 python tools/reduce_probe.py > gpurun_out/${TAG}_train_torch_ops.txt 2> gpurun_out/${TAG}_probe.err
