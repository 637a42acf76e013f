#!/bin/bash
# Round artefacts on the GPU box: GPU tests, the default bench under rocprofv3 kernel-trace/stats,
# and the product GEMM's PMC traffic passes.  Copy-out: see DESIGN.md "Profiles".
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
rm -rf gpurun_out/prof_bench gpurun_out/pmc_gemm
bash tools/pmc_gemm.sh || { echo "pmc failed"; exit 1; }
bash tools/prof_bench.sh || { echo "prof failed"; tail gpurun_out/prof_bench.err; exit 1; }
cat gpurun_out/prof_bench.json
