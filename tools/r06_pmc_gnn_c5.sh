#!/bin/bash
# round 6: PMC of the GNN layers at C5 (n = 512) with and without the Hilbert block order
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
rm -rf gpurun_out/pmc_c5_ord0 gpurun_out/pmc_c5_ord1
FPM_GNN_ORDER=0 BENCH_ARGS="--config c5" bash tools/pmc_kernel.sh "gnn_layer_kernel" gpurun_out/pmc_c5_ord0 || { echo "pmc ord0 failed"; exit 1; }
FPM_GNN_ORDER=1 BENCH_ARGS="--config c5" bash tools/pmc_kernel.sh "gnn_layer_kernel" gpurun_out/pmc_c5_ord1 || { echo "pmc ord1 failed"; exit 1; }
echo done
