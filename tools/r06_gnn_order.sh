#!/bin/bash
# round 6: GNN graph-2 block order (Hilbert, boxes over 256) -- tests, kernel timing, C5 A/B
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "block_order or n512 or c5 or stream" -v --timeout 250 --timeout-method thread > gpurun_out/r06_order_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_order_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_order_tests.log
B=64 N=512 timeout -k 10 250 python tools/gnn_order_bench.py || exit 1
for v in 0 1 0 1; do
  FPM_GNN_ORDER=$v timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-selfcheck > gpurun_out/r06_c5_ord$v.json 2> gpurun_out/r06_c5_ord$v.err || { tail -5 gpurun_out/r06_c5_ord$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_c5_ord$v.json'));print('order=$v', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']))"
done
