#!/bin/bash
# PMC passes on the 17-channel GNN layer (tools/gnn_bench.py incl. the phase-split launches)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pmc_gnn2; mkdir -p $O
p() { local n=$1; shift; GNN_PHASES=1 timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "gnn_layer_kernel<17" -d $O/$n -o run --output-format csv -- python tools/gnn_bench.py > $O/$n.log 2>&1; }
p sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE && \
p sq2 SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD && \
p mem FETCH_SIZE TCC_HIT_sum && p mem2 WRITE_SIZE TCC_MISS_sum
