#!/bin/bash
# Round 5: kernel traces for the wall-time split (tools/busy_timeline.py): the 128-pair one-chunk
# forward, the default two-stream C3 forward and the same forward on one stream (FPM_STREAMS=1).
#   TAG=r05c bash tools/r05_prof.sh
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05c}
B="--no-cpu-baseline --no-f32-line --no-selfcheck --no-share-line --no-config-lines"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_b128 -o run --output-format csv -- \
  python bench.py --batch 128 --steps 20 --warmup 2 $B > gpurun_out/prof_${tag}_b128.json 2> gpurun_out/prof_${tag}_b128.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c3 -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 1 $B > gpurun_out/prof_${tag}_c3.json 2> gpurun_out/prof_${tag}_c3.err || exit 1
FPM_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c3s1 -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 1 $B > gpurun_out/prof_${tag}_c3s1.json 2> gpurun_out/prof_${tag}_c3s1.err || exit 1
for v in b128 c3 c3s1; do
  python tools/busy_timeline.py gpurun_out/prof_${tag}_$v/run_kernel_trace.csv --gap-ms 0.8 --skip 2 > gpurun_out/${tag}_${v}_timeline.txt 2>&1
done
