#!/bin/bash
# Round 4: gate-passing fast mode (bf16 SplineConv + bf16x3 AFA-U) -- new tests, then an A/B of the
# default bench against the bf16s AFA-U mode (alternating runs).
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "x3out or gated or tail_vs or match_classifier_vs" \
    tests/test_lsa_async.py tests/test_sharded.py > gpurun_out/r04a_tests.log 2>&1
i=0
for m in bf16x3 bf16s bf16x3 bf16s; do
    i=$((i + 1))
    FPM_AFAU_DTYPE=$m timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line \
        --no-share-line --no-selfcheck > gpurun_out/r04a_bench_${i}_$m.json 2>> gpurun_out/r04a_bench.err
done
