#!/bin/bash
# run selected GPU test files (args), verbose, each under its own time limit
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest "$@" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || { tail -60 gpurun_out/quick_tests.log; exit 1; }
tail -15 gpurun_out/quick_tests.log
