#!/bin/bash
# round 4: combine residency-cap A/B (kernel trace) + GNN layer phase split
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V="combine_lds_kb=0 combine_lds_kb=24 combine_lds_kb=40 combine_lds_kb=56 combine_npb=8 combine_npb=16"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/cb -o run --output-format csv -- python tools/combine_bench.py $V > gpurun_out/r04h_cb.log 2>&1 || { tail gpurun_out/r04h_cb.log; exit 1; }
python tools/combine_bench.py --parse gpurun_out/cb $V > gpurun_out/r04h_combine_ab.txt
GNN_PHASES=1 timeout -k 10 300 python tools/gnn_bench.py > gpurun_out/r04h_gnn_phases.txt 2>&1
