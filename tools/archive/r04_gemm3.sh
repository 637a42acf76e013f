#!/bin/bash
# round 4: 3-stage 256x128 GEMM + fast softplus -- tests, then a kernel trace of the bench command
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "gemm or afau or gated or x3out or affinity or n256_parity or c2_parity" > gpurun_out/r04g_tests.log 2>&1
TAG=r04g bash tools/prof_bench.sh r04g
f=$(find gpurun_out/prof_r04g -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r04g_bench_kernel_stats.csv
python tools/kstats.py gpurun_out/r04g_bench_kernel_stats.csv 12 24 > gpurun_out/r04g_kstats.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line --no-selfcheck > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err
