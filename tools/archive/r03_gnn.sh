#!/bin/bash
# GNN-layer check: kernel tests, then the isolated layer timing per grouping
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r03g}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "gnn or forward_n256 or c2 or c4" > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -8 gpurun_out/${tag}_tests.log; [ $rc -eq 0 ] || exit $rc
GNN_PHASES=1 timeout -k 10 200 python tools/gnn_bench.py > gpurun_out/${tag}_bench.txt 2>&1; rc=$?
cat gpurun_out/${tag}_bench.txt; exit $rc
