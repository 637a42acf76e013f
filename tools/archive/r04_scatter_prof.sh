#!/bin/bash
# round 4: combine_scatter_bwd_kernel time with / without the fp32 cell-row writes (kernel trace)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r04af}
for v in 0 1 0 1; do
  FPM_SCATTER_F32_ROWS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sc$v -o run --output-format csv -- python tools/train_bench.py --steps 3 --warmup 1 --cpu-pairs 0 > gpurun_out/prof_sc$v.log 2>&1 || { tail -20 gpurun_out/prof_sc$v.log; exit 1; }
  f=$(find gpurun_out/prof_sc$v -name "*kernel_stats.csv" | head -1)
  echo "FPM_SCATTER_F32_ROWS=$v" >> gpurun_out/${TAG}_scatter_kernel.txt
  grep -E "combine_scatter_bwd|\"Name\"" "$f" >> gpurun_out/${TAG}_scatter_kernel.txt
  rm -rf gpurun_out/prof_sc$v
done
cat gpurun_out/${TAG}_scatter_kernel.txt
