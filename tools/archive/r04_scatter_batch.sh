#!/bin/bash
# round 4: scatter SplineConv backward with out-edge load batches (FPM_SCATTER_BATCH 4) vs one edge
# at a time (1): training GPU tests, then the kernel's time per launch (kernel trace), interleaved
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r04ag}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train.py -m gpu \
    > gpurun_out/${TAG}_train_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_train_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_train_tests.log
for v in 1 4 1 4; do
  FPM_SCATTER_BATCH=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sb$v -o run --output-format csv -- python tools/train_bench.py --steps 3 --warmup 1 --cpu-pairs 0 > gpurun_out/prof_sb$v.log 2>&1 || { tail -20 gpurun_out/prof_sb$v.log; exit 1; }
  f=$(find gpurun_out/prof_sb$v -name "*kernel_stats.csv" | head -1)
  echo "FPM_SCATTER_BATCH=$v" >> gpurun_out/${TAG}_scatter_batch.txt
  grep -E "combine_scatter_bwd|\"Name\"" "$f" >> gpurun_out/${TAG}_scatter_batch.txt
  grep -E "^\{" gpurun_out/prof_sb$v.log >> gpurun_out/${TAG}_scatter_batch.txt || true
  rm -rf gpurun_out/prof_sb$v
done
cat gpurun_out/${TAG}_scatter_batch.txt
