#!/bin/bash
# same-box A/B of the default bench: in-tree library vs the previous commit's build
# (tools/_ab/libfpm_prev.so), alternating; first the op tests of the changed kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "topk or gated or batch_vs_solo" > gpurun_out/r04aa_tests.log 2>&1 || { tail -30 gpurun_out/r04aa_tests.log; exit 1; }
tail -1 gpurun_out/r04aa_tests.log
for lib in prev cur prev cur prev cur; do
  if [ $lib = prev ]; then export FPM_LIB_PATH=$PWD/tools/_ab/libfpm_prev.so; else unset FPM_LIB_PATH; fi
  timeout -k 10 400 python bench.py --no-selfcheck --no-cpu-baseline --no-f32-line --no-share-line > gpurun_out/r04aa_bench_$lib.json 2>> gpurun_out/r04aa_ab.err || { tail -20 gpurun_out/r04aa_ab.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/r04aa_bench_$lib.json').read().strip().splitlines()[-1])
print('$lib', round(d['value']), round(d['ms_per_step'],2), d.get('gpu_stage_pairs_per_s'))" >> gpurun_out/r04aa_ab.txt
done
cat gpurun_out/r04aa_ab.txt
