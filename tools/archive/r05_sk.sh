#!/bin/bash
# Round 5: L-form Sinkhorn vector tile I/O + soft top-k one-fma fast pass: tests, per-launch timing,
# PMC (VALU per wave) of both kernels, then the default bench.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_train.py tests/test_ref_ops.py -m gpu -x -v \
  --timeout 240 --timeout-method thread -k "sinkhorn or topk or soft or gated or n256 or bitwise or lform or c1 or ragged or n512" \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
for b in 32 128; do B=$b timeout -k 10 120 python tools/topk_ab.py > gpurun_out/${tag}_topk_ab_b$b.txt 2>&1 || exit 1; done
timeout -k 10 120 python tools/sk_steps.py > gpurun_out/${tag}_sk_steps.txt 2>&1 || exit 1
bash tools/pmc_kernel.sh "sinkhorn_lform|soft_topk" gpurun_out/pmc_$tag || { tail gpurun_out/pmc_$tag/*.log; exit 1; }
python tools/pmc_table.py gpurun_out/pmc_$tag gpurun_out/pmc_${tag}.json > gpurun_out/pmc_${tag}.txt
timeout -k 10 400 python bench.py --no-config-lines > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
python - <<'PY'
import json,os
tag=os.environ.get("TAG","r05h")
d=json.load(open("gpurun_out/%s_bench.json"%tag))
s=d["share128_line"]
print(round(d["value"]), round(d["gpu_stage_pairs_per_s"]), "share128", round(s["value"]), round(s["gpu_stage_pairs_per_s"]), d["parity_gate"]["passed"], d["parity_gate"]["max_abs"], d["timed_batch_selfcheck"])
PY
