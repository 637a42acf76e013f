#!/bin/bash
# PMC passes on one kernel family of a short single-stream bench run:
#   bash tools/pmc_kernel.sh <kernel-regex> <outdir>
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
RE="$1"; OUT="$2"
mkdir -p "$OUT"
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  FPM_STREAMS=1 timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" -d "$OUT/$name" -o run \
    --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/$name.log" 2>&1
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU &&
run mem FETCH_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE &&
run mem2 WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_SALU
