#!/bin/bash
# rocprofv3 kernel trace of the 128-pairs-per-GPU forward (BASELINE's global batch over 8 GPUs):
#   bash tools/prof_b128.sh <tag>   -> gpurun_out/prof_<tag>/ (+ .json / .err)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-b128}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python bench.py --batch 128 --steps 20 --warmup 2 --no-cpu-baseline --no-f32-line --no-selfcheck --no-share-line \
  > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
