#!/bin/bash
# PMC passes on the AFA-U attention microbenchmark (tools/attn_bench.py): bash tools/pmc_attn.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT="$1"; mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex afau_row_attn -d "$OUT/$name" -o run \
    --output-format csv -- python tools/attn_bench.py > "$OUT/$name.log" 2>&1
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU &&
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
