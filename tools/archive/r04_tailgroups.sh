#!/bin/bash
# share-128 line vs one-chunk tail groups (FPM_TAIL_GROUPS 4 = default vs 6 / 8), interleaved on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for g in 4 8 6 4 8 6; do
  FPM_TAIL_GROUPS=$g timeout -k 10 400 python bench.py --no-selfcheck --no-cpu-baseline --no-f32-line > gpurun_out/r04y_b.json 2>> gpurun_out/r04y_ab.err || { tail -20 gpurun_out/r04y_ab.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r04y_b.json').read().strip().splitlines()[-1])
s=d.get('share128_line') or {}
print('groups=$g', 'C3', round(d['value']), '| share128', round(s.get('value', 0)), s.get('ms_per_step'), s.get('gpu_stage_pairs_per_s'), s.get('host_lsa_ms'))" >> gpurun_out/r04y_ab.txt
done
cat gpurun_out/r04y_ab.txt
