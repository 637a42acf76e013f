#!/bin/bash
# streaming Sinkhorn per-launch timing only (both layouts, 2 / 20 steps, RW 1 vs 4)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rw in ${RWS:-1 4}; do for it in 2 20; do for t in n t; do
  FPM_SK_STREAM_RW=$rw timeout -k 10 120 python tools/sk_stream_bench.py 128 512 $it $t || exit 1
done; done; done
