#!/bin/bash
# training-step bench + kernel stats of it (rocprofv3 kernel trace)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/train_bench.py "$@" > gpurun_out/train_bench.json 2> gpurun_out/train_bench.err || { tail -30 gpurun_out/train_bench.err; exit 1; }
cat gpurun_out/train_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --steps 2 --warmup 1 --cpu-pairs 0 "$@" > gpurun_out/prof_train.log 2>&1 || { tail -20 gpurun_out/prof_train.log; exit 1; }
f=$(find gpurun_out/prof_train -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/train_kernel_stats.csv
python tools/kstats.py gpurun_out/train_kernel_stats.csv 3 30
