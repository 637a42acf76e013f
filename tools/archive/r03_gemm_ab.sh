#!/bin/bash
# C3 A/B of the SplineConv product GEMM kernel (gemm_phase 1: 256x256 phase kernel, one workgroup
# per CU; 2: 128x128 generic kernel, two per CU), each twice; then the host timeline.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
k=0
for rep in 1 2; do for v in 1 2; do
  k=$((k+1))
  timeout -k 10 200 python bench.py --steps 15 --warmup 2 --no-cpu-baseline --no-f32-line --no-selfcheck --tuning gemm_phase=$v > gpurun_out/gab$k.json 2> gpurun_out/gab$k.err || { tail gpurun_out/gab$k.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/gab$k.json'))
sl=d.get('share128_line') or {}; r=d['roofline']; p=d.get('parity_vs_oracle') or {}
print('[gemm_phase=$v]', round(d['value']), 'gpu-stage', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d['host_lsa_ms_per_step'],1), 'share128', round(sl.get('value', 0)), 'gemm ms', round(r['avg_launch_ms'],3), 'iso', round(r['isolated_avg_launch_ms'],3), 'parity', {k: p.get(k) for k in ('ds_mat_max_abs', 'perm_classes') if k in p})"
done; done
timeout -k 10 200 python tools/timeline.py 1024 > gpurun_out/timeline1024.txt 2>&1; grep -v amdgpu.ids gpurun_out/timeline1024.txt
timeout -k 10 200 python tools/timeline.py 128 > gpurun_out/timeline128.txt 2>&1; grep -v amdgpu.ids gpurun_out/timeline128.txt
