#!/bin/bash
# round 4: one-chunk tail groups -- tests, then the 128-pair share line A/B (FPM_TAIL_GROUPS 1 vs 4)
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "tail_groups or affinity_fwd or device_tail" > gpurun_out/r04d_tests.log 2>&1
i=0
for g in 1 4 1 4; do
    i=$((i + 1))
    FPM_TAIL_GROUPS=$g timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line \
        --no-selfcheck > gpurun_out/r04d_bench_${i}_g$g.json 2>> gpurun_out/r04d_bench.err
done
