#!/bin/bash
# round 6: the 2-workgroups-per-CU product GEMM (gemm_pp.h) vs the phase kernel -- micro-benchmark
# (bit-identity + isolated rate), then the C3 bench with each (same box, interleaved)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemm_bench > gpurun_out/r06_gemm_pp_micro.txt 2>&1 || { cat gpurun_out/r06_gemm_pp_micro.txt; exit 1; }
cat gpurun_out/r06_gemm_pp_micro.txt
for pp in 0 1 0 1; do
  FPM_GEMM_PP=$pp timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --no-selfcheck > gpurun_out/r06_pp$pp.json 2> gpurun_out/r06_pp$pp.err || { tail -20 gpurun_out/r06_pp$pp.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06_pp$pp.json'));r=d['roofline'];print('pp=$pp', round(d['value']), 'pairs/s', 'gemm avg ms %.3f'%r['avg_launch_ms'], 'iso ms %.3f'%r['isolated_avg_launch_ms'], 'exec_frac %.3f'%r['exec_frac'])"
done
