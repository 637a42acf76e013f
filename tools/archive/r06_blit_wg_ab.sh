#!/bin/bash
# round 6: ds_mat D2H blit kernel size (DEBUG_CLR_LIMIT_BLIT_WG) at C3
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in default 4 64 default 4 64; do
  if [ $v = default ]; then E=""; else E="DEBUG_CLR_LIMIT_BLIT_WG=$v"; fi
  env $E timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --parity-pairs 0 > gpurun_out/r06_bw_$v.json 2> gpurun_out/r06_bw_$v.err || { tail -5 gpurun_out/r06_bw_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_bw_$v.json'));print('blit_wg=$v', round(d['value']), 'gpu', round(d['gpu_stage_pairs_per_s']))"
done
