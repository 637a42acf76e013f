#!/bin/bash
# Round 5: near-fp32 Kp operands in the bf16 mode: gated-mode / parity / bit-identity GPU tests,
# then the default bench with and without the split operands (FPM_KP_X3=0), interleaved.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r05d}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_frontend.py tests/test_batch.py -m gpu -x -v \
  --timeout 240 --timeout-method thread -k "gated or image or bitwise or n256 or probe or sharded or chunk or bf16" \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 400 python bench.py --no-config-lines > gpurun_out/${tag}_bench_x3.json 2> gpurun_out/${tag}_bench_x3.err || exit 1
FPM_KP_X3=0 timeout -k 10 300 python bench.py --no-config-lines --no-cpu-baseline --no-f32-line > gpurun_out/${tag}_bench_plain.json 2> gpurun_out/${tag}_bench_plain.err || exit 1
timeout -k 10 300 python bench.py --no-config-lines --no-cpu-baseline --no-f32-line > gpurun_out/${tag}_bench_x3b.json 2> gpurun_out/${tag}_bench_x3b.err || exit 1
python - <<'PY'
import json,os
tag=os.environ.get("TAG","r05d")
for v in ("x3","plain","x3b"):
    d=json.load(open("gpurun_out/%s_bench_%s.json"%(tag,v)))
    print(v, round(d["value"]), round(d["gpu_stage_pairs_per_s"]), round(d["share128_line"]["value"]), d["parity_gate"] and d["parity_gate"]["max_abs"], d["parity_gate"] and d["parity_gate"]["passed"])
PY
