#!/bin/bash
# single-stream kernel-trace stats of the bench (true per-kernel durations, no co-running stream):
#   TAG=<tag> bash tools/prof_1s.sh [bench args]   -> gpurun_out/prof1s_<tag>_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r03}
FPM_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1s_$tag -o run --output-format csv -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-line --no-selfcheck "$@" > gpurun_out/prof1s_$tag.log 2>&1 || { tail -20 gpurun_out/prof1s_$tag.log; exit 1; }
f=$(find gpurun_out/prof1s_$tag -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/prof1s_${tag}_kernel_stats.csv
python tools/kstats.py gpurun_out/prof1s_${tag}_kernel_stats.csv 8 30
