#!/bin/bash
# round 6: C5 (n = 512: a pair's 17-channel slab is 17.8 MB) -- GNN phase-1 channel-group sweeps 1 / 2 / 3
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in 1 2 3 1 2 3; do
  timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-selfcheck --tuning gnn_sweeps=$v > gpurun_out/r06_c5_sw$v.json 2> gpurun_out/r06_c5_sw$v.err || { tail -5 gpurun_out/r06_c5_sw$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_c5_sw$v.json'));print('sweeps=$v', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']), 'gate', (d.get('parity_gate') or {}).get('passed'))"
done
