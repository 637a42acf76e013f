#!/bin/bash
# GNN phase-1 channel-group sweeps: bit-identity test, then the default bench with gnn_sweeps 1 / 2 / 3
# alternating on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "sweeps" > gpurun_out/r04w_tests.log 2>&1 || { tail -30 gpurun_out/r04w_tests.log; exit 1; }
for v in 1 2 3 1 2 3; do
  timeout -k 10 400 python bench.py --no-selfcheck --no-cpu-baseline --no-f32-line --no-share-line --tuning gnn_sweeps=$v > gpurun_out/r04w_b.json 2>> gpurun_out/r04w_ab.err || { tail -20 gpurun_out/r04w_ab.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r04w_b.json').read().strip().splitlines()[-1])
print('sweeps=$v', round(d['value']), round(d['ms_per_step'],2), d.get('gpu_stage_pairs_per_s'))" >> gpurun_out/r04w_ab.txt
done
cat gpurun_out/r04w_ab.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w2 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-selfcheck --no-cpu-baseline --no-f32-line --no-share-line --parity-pairs 0 --tuning gnn_sweeps=2 > gpurun_out/prof_w2.log 2>&1 || true
