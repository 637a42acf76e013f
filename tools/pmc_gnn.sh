#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pmc_gnn2; mkdir -p $O
p() { local n=$1; shift; timeout -k 10 180 rocprofv3 --pmc "$@" --kernel-include-regex "gnn_layer_kernel<17>" -d $O/$n -o run --output-format csv -- python tools/gnn_bench.py > $O/$n.log 2>&1; }
p a FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY && p b WRITE_SIZE TCC_HIT_sum TCC_MISS_sum && p c SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
