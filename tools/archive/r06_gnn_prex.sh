#!/bin/bash
# round 6: GNN layer with the point's channels prefetched before phase 1 (gnn_prefetch_x) -- bit
# identity, isolated timing, C3 A/B
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "variants_bit_identical or gnn" -v --timeout 200 --timeout-method thread > gpurun_out/r06_prex_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06_prex_tests.log | tail; exit 1; }
grep -cE "PASSED" gpurun_out/r06_prex_tests.log
timeout -k 10 200 python tools/gnn_bench.py "gnn_prefetch_x=0" "gnn_prefetch_x=1" || exit 1
for v in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --parity-pairs 0 --tuning gnn_prefetch_x=$v > gpurun_out/r06_prex_$v.json 2> gpurun_out/r06_prex_$v.err || { tail -5 gpurun_out/r06_prex_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_prex_$v.json'));print('prex=$v', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']))"
done
