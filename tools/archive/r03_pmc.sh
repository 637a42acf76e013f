#!/bin/bash
# round-3 profile set: kernel traces (two-stream bench + single-stream), PMC of the main kernels,
# PMC HBM traffic of the product GEMM
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r03i}
bash tools/r03_prof.sh > gpurun_out/${tag}_prof.txt 2>&1 || { tail -20 gpurun_out/${tag}_prof.txt; exit 1; }
head -32 gpurun_out/${tag}_prof.txt
bash tools/pmc_kernel.sh "gnn_layer_kernel|afau_row_attn_v|sinkhorn_reg|combine_kernel|plan_multi|soft_topk_kernel" gpurun_out/pmc_$tag || { tail gpurun_out/pmc_$tag/*.log; exit 1; }
python tools/pmc_table.py gpurun_out/pmc_$tag gpurun_out/pmc_${tag}.json > gpurun_out/pmc_${tag}.txt; cat gpurun_out/pmc_${tag}.txt
bash tools/pmc_gemm.sh && echo pmc_gemm done
