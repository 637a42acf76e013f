#!/bin/bash
# Round 5: small-batch tail (attention head split, coefficient kernel): tests, then bench A/B
# (afau_head_split forced 1 = the round-4 launch shape vs the default by-size split), interleaved.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_batch.py tests/test_sharded.py -m gpu -x -v \
  --timeout 240 --timeout-method thread -k "attn or gated or bitwise or n256 or sharded or chunk or affinity or smoke or c1" \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
B="--no-config-lines --no-cpu-baseline --no-f32-line"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/${tag}_new$i.json 2> gpurun_out/${tag}_new$i.err || exit 1
  timeout -k 10 300 python bench.py $B --tuning afau_head_split=1 > gpurun_out/${tag}_old$i.json 2> gpurun_out/${tag}_old$i.err || exit 1
done
python - <<'PY'
import json,os
tag=os.environ.get("TAG","r05f")
for v in ("new1","old1","new2","old2"):
    d=json.load(open("gpurun_out/%s_%s.json"%(tag,v)))
    s=d["share128_line"]
    print(v, round(d["value"]), round(d["gpu_stage_pairs_per_s"]), "share128", round(s["value"]), round(s["gpu_stage_pairs_per_s"]), round(s["host_lsa_ms_per_step"],2), round(s["enqueue_ms"],2))
PY
