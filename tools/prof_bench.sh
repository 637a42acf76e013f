#!/bin/bash
# rocprofv3 kernel-trace + stats of the default bench command (the round's committed profile)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 1 --cpu-pairs 8 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
