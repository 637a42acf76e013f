#!/bin/bash
# default bench (graph-build field) + single-stream kernel-trace stats (true per-kernel durations)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-pairs 4 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; grep "graph build\|step:" gpurun_out/bench.err | tail -3
FPM_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1s -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_1s.log 2>&1 || { tail -20 gpurun_out/prof_1s.log; exit 1; }
find gpurun_out/prof_1s -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_1s_kernel_stats.csv
echo done
