#!/bin/bash
# round 4: fused train-mode MatchClassifier -- its parity tests, then the training step A/B (MIOpen
# composition vs fused) and the fused step's kernel stats
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r04l}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train.py \
    -k "match_cls_train or bn_relu or weight_pack or outer_sum or gnn or afau or train_step" > gpurun_out/${TAG}_cls_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_cls_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_cls_tests.log
for cfg in "FPM_CLS_TRAIN=fused" "FPM_AFAU_TRAIN_X3=0" "FPM_CLS_TRAIN=torch" "FPM_CLS_TRAIN=fused" "FPM_AFAU_TRAIN_X3=0" "FPM_CLS_TRAIN=torch"; do
  env $cfg timeout -k 10 300 python tools/train_bench.py --cpu-pairs 0 >> gpurun_out/${TAG}_cls_ab.txt 2>> gpurun_out/${TAG}_cls_ab.err || { tail -30 gpurun_out/${TAG}_cls_ab.err; exit 1; }
  echo "cfg=$cfg" >> gpurun_out/${TAG}_cls_ab.txt
done
cat gpurun_out/${TAG}_cls_ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cls -o run --output-format csv -- python tools/train_bench.py --steps 2 --warmup 1 --cpu-pairs 0 > gpurun_out/prof_cls.log 2>&1 || { tail -20 gpurun_out/prof_cls.log; exit 1; }
f=$(find gpurun_out/prof_cls -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_train_kernel_stats.csv
python tools/kstats.py gpurun_out/${TAG}_train_kernel_stats.csv 3 40 > gpurun_out/${TAG}_train_kstats.txt
