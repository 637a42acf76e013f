#!/bin/bash
# Round 5, final tree: the profile set (two-stream kernel trace of the bench command + roofline
# table, PMC of the main kernels, product-GEMM HBM traffic) and the image-path k_prob diagnostic.
#   TAG=r05z bash tools/r05_prof_final.sh
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05z}
TAG=$tag bash tools/r04_prof.sh > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
timeout -k 10 300 python tools/kprob_gpu_diag.py --json gpurun_out/${tag}_kprob_gpu.json > gpurun_out/${tag}_kprob_gpu.txt 2>&1 || { tail gpurun_out/${tag}_kprob_gpu.txt; exit 1; }
tail -3 gpurun_out/${tag}_kprob_gpu.txt
head -12 gpurun_out/${tag}_kstats.txt
