#!/bin/bash
# PMC passes on the 17-channel GNN layer kernel (tools/gnn_bench.py, B=128, n=256)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pmc_gnn; mkdir -p $O
p() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "gnn_layer_kernel<17" -d $O/$n -o run --output-format csv -- python tools/gnn_bench.py > $O/$n.log 2>&1; }
p a FETCH_SIZE GRBM_GUI_ACTIVE && p b WRITE_SIZE TCC_HIT_sum TCC_MISS_sum && p c SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY
for n in a b c; do f=$(find $O/$n -name "*counter_collection.csv" | head -1); python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print("%-22s mean per launch %.4g  (%d launches)" % (k, sum(v) / len(v), len(v)))
PY
done
