#!/bin/bash
# Round 5: zero-copy ds_mat (soft top-k writes the pinned rows) vs the copy-stream D2H: bitwise test,
# then interleaved bench runs FPM_ZERO_COPY = 0 / 1 / 2 (headline + 128-pair share line).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05g}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "zero_copy or tail_groups or batch_vs_solo" > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
B="--no-config-lines --no-cpu-baseline --no-f32-line"
for i in 1 2; do
  for z in 0 1 2; do
    FPM_ZERO_COPY=$z timeout -k 10 300 python bench.py $B > gpurun_out/${tag}_z${z}_$i.json 2> gpurun_out/${tag}_z${z}_$i.err || exit 1
  done
done
python - <<'PY'
import json,os
tag=os.environ.get("TAG","r05g")
for i in (1,2):
    for z in (0,1,2):
        d=json.load(open("gpurun_out/%s_z%d_%d.json"%(tag,z,i)))
        s=d["share128_line"]
        print("z%d run%d"%(z,i), round(d["value"]), round(d["gpu_stage_pairs_per_s"]), "lsa", round(d["host_lsa_ms_per_step"],2), "share128", round(s["value"]), round(s["gpu_stage_pairs_per_s"]), round(s["host_lsa_ms_per_step"],2), d["timed_batch_selfcheck"])
PY
