#!/bin/bash
# round 4: Sinkhorn L-form epilogue change -- parity tests, the per-step probe, one default bench
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r04o}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_train.py \
    -k "sinkhorn or gated or soft_topk" > gpurun_out/${TAG}_sk_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_sk_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_sk_tests.log
timeout -k 10 300 python tools/sk_steps.py 1024 256 > gpurun_out/${TAG}_sk_steps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_sk_steps.txt; exit 1; }
cat gpurun_out/${TAG}_sk_steps.txt
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
