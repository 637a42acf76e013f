#!/bin/bash
# Round 5: run-to-run spread of the default C3 forward (separate processes), new stream layout vs the
# round-4 one (FPM_PROLOGUE_FORK=0 FPM_STAGEC_STREAM=0)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05m}
B="--no-config-lines --no-cpu-baseline --no-f32-line --no-share-line --no-selfcheck --steps 10"
for i in 1 2 3 4; do
  timeout -k 10 200 python bench.py $B > gpurun_out/${tag}_new$i.json 2> gpurun_out/${tag}_new$i.err || exit 1
  FPM_PROLOGUE_FORK=0 timeout -k 10 200 python bench.py $B > gpurun_out/${tag}_old$i.json 2> gpurun_out/${tag}_old$i.err || exit 1
done
timeout -k 10 200 python tools/stage_events.py --batch 1024 --reps 2 --timeline > gpurun_out/${tag}_timeline_c3.txt 2>&1 || exit 1
for f in gpurun_out/${tag}_new?.err gpurun_out/${tag}_old?.err; do echo "$f $(grep streams: $f | cut -c1-200)"; done
python - <<'PY'
import json,os
tag=os.environ.get("TAG","r05m")
for v in ("new","old"):
    print(v, [ (round(json.load(open("gpurun_out/%s_%s%d.json"%(tag,v,i)))["value"]), round(json.load(open("gpurun_out/%s_%s%d.json"%(tag,v,i)))["gpu_stage_pairs_per_s"])) for i in (1,2,3,4)])
PY
