#!/bin/bash
# Round 5, final tree: the driver's three commands (full GPU test suite, smoke, default bench).
#   TAG=r05z bash tools/r05_final.sh
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05z}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python - <<'PY'
import json, os
tag = os.environ.get("TAG", "r05z")
d = json.load(open("gpurun_out/%s_bench.json" % tag))
s = d["share128_line"]
print("C3", round(d["value"]), "gpu", round(d["gpu_stage_pairs_per_s"]), "share128", round(s["value"]), round(s["gpu_stage_pairs_per_s"]),
      "gate", d["parity_gate"]["passed"], d["parity_gate"]["max_abs"], "selfcheck", d["timed_batch_selfcheck"])
for k in ("c2_line", "c4_line", "c5_line", "train_line"):
    v = d.get(k) or {}
    print(k, round(v.get("value", 0)), (v.get("parity_gate") or {}).get("passed"))
print("roofline", d["roofline"])
PY
