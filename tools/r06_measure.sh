#!/bin/bash
# Round-6 measurement pass on the GPU box: GPU tests, smoke, the default bench (all config lines), the
# bench under rocprofv3 kernel-trace/stats, the product GEMM's PMC traffic passes and per-kernel PMC
# passes (single stream).  Outputs under gpurun_out/r06m_*; copied into profiles/ afterwards.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-r06m}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));print('bench', round(d['value']), d['ms_per_step'], d['parity_gate']['passed'], d['roofline']['frac'], d['roofline']['exec_frac'])"
rm -rf gpurun_out/pmc_gemm gpurun_out/prof_$T gpurun_out/pmc_$T
bash tools/pmc_gemm.sh || { echo "pmc_gemm failed"; exit 1; }
bash tools/prof_bench.sh $T || { echo "prof failed"; tail gpurun_out/prof_$T.err; exit 1; }
bash tools/pmc_kernel.sh "gemm_phase|combine_kernel|gnn_layer_kernel|sinkhorn_lform|soft_topk_kernel|afau_row_attn|gemm_big_kernel" gpurun_out/pmc_$T || { echo "pmc_kernel failed"; exit 1; }
echo done
