#!/bin/bash
# round-4: profile set (tools/r04_prof.sh) then the training torch-op attribution probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r04c} bash tools/r04_prof.sh > gpurun_out/${TAG:-r04c}_prof.log 2>&1 || exit 1
timeout -k 10 300 python tools/reduce_probe.py > gpurun_out/r04_train_torch_ops.txt 2> gpurun_out/r04_train_torch_ops.err
