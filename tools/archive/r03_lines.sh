#!/bin/bash
# C2 / C4 / C5 bench lines and the training step of the round-3 tree
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in c2 c4 c5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line > gpurun_out/r03_${c}_bench.json 2> gpurun_out/r03_${c}_bench.err || { tail -20 gpurun_out/r03_${c}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03_${c}_bench.json')); print('$c', round(d['value']), 'gpu-stage', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d['host_lsa_ms_per_step'],1))"
done
timeout -k 10 300 python tools/train_bench.py > gpurun_out/r03_train_bench.json 2> gpurun_out/r03_train_bench.err || { tail -30 gpurun_out/r03_train_bench.err; exit 1; }
cat gpurun_out/r03_train_bench.json
