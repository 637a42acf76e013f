#!/bin/bash
# C3 bench under alternating environment settings, each run twice:
#   bash tools/env_ab.sh "" "FPM_COPY_KIND=1024" "DEBUG_CLR_LIMIT_BLIT_WG=16"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
k=0
for rep in 1 2; do for cfg in "$@"; do
  k=$((k+1))
  env $cfg timeout -k 10 200 python bench.py --steps ${STEPS:-15} --warmup 2 --no-cpu-baseline --no-f32-line --no-selfcheck ${BENCH_ARGS} > gpurun_out/envab$k.json 2> gpurun_out/envab$k.err || { tail gpurun_out/envab$k.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/envab$k.json'))
sl=d.get('share128_line') or {}; r=d.get('roofline') or {}
print('[$cfg]', round(d['value']), 'gpu-stage', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d['host_lsa_ms_per_step'],1), 'ms', round(d['ms_per_step'],2), 'share128', round(sl.get('value', 0)), sl.get('chunks'), 'gemm ms', round(r.get('avg_launch_ms') or 0, 3), 'iso', round(r.get('isolated_avg_launch_ms') or 0, 3))"
done; done
