#!/bin/bash
# SDMA ds_mat hand-off: GPU tests of the copy and the forward, then C3 A/B blit vs dma (each twice)
# and a kernel trace of the dma mode.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "dma or graph_replay or side_streams" > gpurun_out/dma_tests.log 2>&1 || { tail -30 gpurun_out/dma_tests.log; exit 1; }
tail -2 gpurun_out/dma_tests.log
k=0
for rep in 1 2; do for v in blit dma; do
  k=$((k+1))
  FPM_D2H=$v timeout -k 10 200 python bench.py --steps 15 --warmup 2 --no-cpu-baseline --no-f32-line --no-selfcheck > gpurun_out/dmaab$k.json 2> gpurun_out/dmaab$k.err || { tail gpurun_out/dmaab$k.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/dmaab$k.json'))
sl=d.get('share128_line') or {}
print('[$v]', round(d['value']), 'gpu-stage', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d['host_lsa_ms_per_step'],1), 'ms', round(d['ms_per_step'],2), 'share128', round(sl.get('value', 0)))"
done; done
for rep in 1 2; do for v in 0 1; do
  FPM_SIDES=$v timeout -k 10 200 python bench.py --batch 128 --steps 30 --warmup 3 --no-cpu-baseline --no-f32-line --no-selfcheck --no-share-line > gpurun_out/sides$v$rep.json 2> gpurun_out/sides$v$rep.err || { tail gpurun_out/sides$v$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/sides$v$rep.json'))
print('[sides=$v] b128', round(d['value']), 'gpu-stage', round(d['gpu_stage_pairs_per_s']), 'lsa_ms', round(d['host_lsa_ms_per_step'],2), 'ms', round(d['ms_per_step'],2))"
done; done
FPM_D2H=dma timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dma -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-f32-line --no-selfcheck --no-share-line > gpurun_out/prof_dma.json 2> gpurun_out/prof_dma.err
timeout -k 10 120 python tools/sk_bench.py > gpurun_out/sk_bench.txt 2>&1; cat gpurun_out/sk_bench.txt
