#!/bin/bash
# round 6: where the 128-pair forward's GPU stage goes -- synchronised stage timing (128 vs 1024
# pairs) and a kernel trace of the 128-pair bench with the busy/idle split
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
[ -n "$SKIP_ST" ] || timeout -k 10 200 python tools/stage_timing.py 128 256 bf16 > gpurun_out/r06_st128.txt 2>&1 || { tail gpurun_out/r06_st128.txt; exit 1; }
[ -n "$SKIP_ST" ] || timeout -k 10 200 python tools/stage_timing.py 1024 256 bf16 > gpurun_out/r06_st1024.txt 2>&1 || { tail gpurun_out/r06_st1024.txt; exit 1; }
[ -n "$SKIP_ST" ] || grep iter gpurun_out/r06_st128.txt gpurun_out/r06_st1024.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof128 -o p128 --output-format csv -- python bench.py --batch 128 --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-share-line --no-config-lines --no-selfcheck > gpurun_out/r06_b128.json 2> gpurun_out/r06_b128.err || { tail gpurun_out/r06_b128.err; exit 1; }
f=$(ls gpurun_out/prof128/*/p128_kernel_trace.csv | head -1)
python tools/busy_timeline.py "$f" --skip 3 --top 20 > gpurun_out/r06_b128_busy.txt && head -60 gpurun_out/r06_b128_busy.txt
s=$(ls gpurun_out/prof128/*/p128_kernel_stats.csv | head -1); cp "$s" gpurun_out/r06_b128_kstats.csv
