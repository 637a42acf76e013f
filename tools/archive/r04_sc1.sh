#!/bin/bash
# round 4: sc1 store-policy A/B (GNN layer, combine, product GEMM) -- bit-identity test, GNN kernel
# microbench, then interleaved bench runs per variant
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "store_cache_policies or affinity_epilogue or n256_parity or c2_parity or gated_mode_c3 or c1_parity" > gpurun_out/r04e_tests.log 2>&1
timeout -k 10 300 python tools/gnn_bench.py gnn_store_sc1=0 gnn_store_sc1=1 > gpurun_out/r04e_gnn_bench.txt 2>&1
for r in 1 2; do
  for v in "gnn_store_sc1=0,combine_store_sc1=0,gemm_store_sc1=0" "gnn_store_sc1=1,combine_store_sc1=1,gemm_store_sc1=1" \
           "gnn_store_sc1=1,combine_store_sc1=0,gemm_store_sc1=0" "gnn_store_sc1=0,combine_store_sc1=1,gemm_store_sc1=0" \
           "gnn_store_sc1=0,combine_store_sc1=0,gemm_store_sc1=1"; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line --no-selfcheck \
        --no-share-line --tuning "$v" >> gpurun_out/r04e_bench.jsonl 2>> gpurun_out/r04e_bench.err
  done
done
