#!/bin/bash
# graph-construction tests + the full GPU suite + bench (development check)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graphs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/graphs_tests.log 2>&1 || { tail -40 gpurun_out/graphs_tests.log; exit 1; }
tail -3 gpurun_out/graphs_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-pairs 8 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; grep "step:" gpurun_out/bench.err | tail -3
