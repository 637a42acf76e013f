#!/bin/bash
# round 6: kernel trace of the synchronised stage-timing forward (one stream, no overlap) at 128 and
# 1024 pairs: isolated per-kernel durations of the small-batch forward
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
N=${N:-256}
for B in ${BS:-128 1024}; do
  FPM_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/st${B}_$N -o st --output-format csv -- python tools/stage_timing.py $B $N bf16 > gpurun_out/st${B}_$N.log 2>&1 || { tail gpurun_out/st${B}_$N.log; exit 1; }
  grep "iter 2" gpurun_out/st${B}_$N.log
done
