#!/bin/bash
# two-stream kernel trace of the bench (committed profile) + single-stream kernel trace
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r03}
bash tools/prof_bench.sh $tag || { tail -20 gpurun_out/prof_$tag.err; exit 1; }
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${tag}_bench_kernel_stats.csv
python tools/kstats.py gpurun_out/${tag}_bench_kernel_stats.csv 12 30
cat gpurun_out/prof_$tag.json | head -c 600; echo
TAG=${tag}1s bash tools/prof_1s.sh
