#!/bin/bash
# training step vs the fpm_gemm 256-wide tile threshold (the SplineConv per-cell weight-gradient
# batches: 468 256-wide tiles) -- FPM_GEMM_BN256_MIN 512 (default) vs 256, interleaved; plus the
# training tests under 256 and the default bench under 256
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
FPM_GEMM_BN256_MIN=256 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train.py -k "spline or train_step" > gpurun_out/r04ab_tests.log 2>&1 || { tail -30 gpurun_out/r04ab_tests.log; exit 1; }
tail -1 gpurun_out/r04ab_tests.log
for v in 512 256 512 256 512 256; do
  FPM_GEMM_BN256_MIN=$v timeout -k 10 300 python tools/train_bench.py --cpu-pairs 0 > gpurun_out/r04ab_t.json 2>> gpurun_out/r04ab.err || { tail -20 gpurun_out/r04ab.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r04ab_t.json').read().strip().splitlines()[-1])
print('bn256_min=$v', round(d['value']), round(d['ms_per_step'], 2))" >> gpurun_out/r04ab_ab.txt
done
for v in 512 256; do
  FPM_GEMM_BN256_MIN=$v timeout -k 10 400 python bench.py --no-selfcheck --no-cpu-baseline --no-f32-line --no-share-line > gpurun_out/r04ab_b.json 2>> gpurun_out/r04ab.err || { tail -20 gpurun_out/r04ab.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r04ab_b.json').read().strip().splitlines()[-1])
print('bench bn256_min=$v', round(d['value']))" >> gpurun_out/r04ab_ab.txt
done
cat gpurun_out/r04ab_ab.txt
