#!/bin/bash
# Sinkhorn L-form round: GPU Sinkhorn parity tests, then C3 A/B over the forward kernel variant
# (sinkhorn_lform 1 / 0 / 2), each twice, then the SDMA probe.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sinkhorn" > gpurun_out/sk_tests.log 2>&1 || { tail -30 gpurun_out/sk_tests.log; exit 1; }
tail -3 gpurun_out/sk_tests.log
k=0
for rep in 1 2; do for v in 1 0 2; do
  k=$((k+1))
  timeout -k 10 200 python bench.py --steps 15 --warmup 2 --no-cpu-baseline --no-f32-line --no-selfcheck --tuning sinkhorn_lform=$v > gpurun_out/skab$k.json 2> gpurun_out/skab$k.err || { tail gpurun_out/skab$k.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/skab$k.json'))
sl=d.get('share128_line') or {}
print('[lform=$v]', round(d['value']), 'gpu-stage', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d['host_lsa_ms_per_step'],1), 'share128', round(sl.get('value', 0)))"
done; done
hipcc --offload-arch=gfx950 -O2 tools/sdma_probe.cpp -lhsa-runtime64 -o gpurun_out/sdma_probe 2>/dev/null && timeout -k 10 120 ./gpurun_out/sdma_probe > gpurun_out/sdma_probe.txt 2>&1; cat gpurun_out/sdma_probe.txt
