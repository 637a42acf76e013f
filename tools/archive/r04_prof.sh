#!/bin/bash
# Round-4 profile set on the current tree: two-stream kernel trace of the bench command (+ roofline
# table), PMC of the main kernels (single stream), PMC HBM traffic of the product GEMM.
#   TAG=r04c bash tools/r04_prof.sh
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r04c}
bash tools/prof_bench.sh $tag || { tail -20 gpurun_out/prof_$tag.err; exit 1; }
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${tag}_bench_kernel_stats.csv
cp gpurun_out/prof_$tag.json gpurun_out/${tag}_bench_under_rocprof.json
python tools/kstats.py gpurun_out/${tag}_bench_kernel_stats.csv 12 30 > gpurun_out/${tag}_kstats.txt
python tools/roofline_table.py gpurun_out/${tag}_bench_kernel_stats.csv --forwards 12 --out gpurun_out/${tag}_roofline_table > gpurun_out/${tag}_roofline.log 2>&1 || true
bash tools/pmc_kernel.sh "gnn_layer_kernel|afau_row_attn_v|sinkhorn_lform|combine_kernel|soft_topk_kernel|gemm_big_kernel<128" gpurun_out/pmc_$tag || { tail gpurun_out/pmc_$tag/*.log; exit 1; }
python tools/pmc_table.py gpurun_out/pmc_$tag gpurun_out/pmc_${tag}.json > gpurun_out/pmc_${tag}.txt
bash tools/pmc_gemm.sh && python tools/pmc_summary.py gpurun_out/pmc_gemm gpurun_out/${tag}_pmc_product_gemm.json > /dev/null && echo pmc_gemm done
