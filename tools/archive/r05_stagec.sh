#!/bin/bash
# Round 5: stage C on its own stream + pinned assignment rows: run-path tests, stage timeline, bench A/B
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_batch.py tests/test_sharded.py tests/test_lsa_async.py -m gpu -x -v \
  --timeout 240 --timeout-method thread -k "bitwise or sharded or chunk or forward or tail or lsa or c1 or n256 or gated or zero_copy" \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 200 python tools/stage_events.py --batch 1024 --reps 2 --timeline > gpurun_out/${tag}_timeline_c3.txt 2>&1 || exit 1
B="--no-config-lines --no-cpu-baseline --no-f32-line"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/${tag}_sc1_$i.json 2> gpurun_out/${tag}_sc1_$i.err || exit 1
  FPM_STAGEC_STREAM=0 timeout -k 10 300 python bench.py $B > gpurun_out/${tag}_sc0_$i.json 2> gpurun_out/${tag}_sc0_$i.err || exit 1
  FPM_PROLOGUE_FORK=0 timeout -k 10 300 python bench.py $B > gpurun_out/${tag}_pf0_$i.json 2> gpurun_out/${tag}_pf0_$i.err || exit 1
  FPM_TAIL_LAST=1.0 timeout -k 10 300 python bench.py $B > gpurun_out/${tag}_tl1_$i.json 2> gpurun_out/${tag}_tl1_$i.err || exit 1
done
python - <<'PY'
import json,os
tag=os.environ.get("TAG","r05l")
for i in (1,2):
    for v in ("sc1","sc0","pf0","tl1"):
        d=json.load(open("gpurun_out/%s_%s_%d.json"%(tag,v,i)))
        s=d["share128_line"]
        print(v, i, round(d["value"]), round(d["gpu_stage_pairs_per_s"]), "ms/step %.2f" % d["ms_per_step"], "share128", round(s["value"]), round(s["gpu_stage_pairs_per_s"]), d["timed_batch_selfcheck"])
PY
