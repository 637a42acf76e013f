set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for z in 1 0 1 0; do FPM_GEMM_PHASE=$z timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ph$z.json 2> gpurun_out/ph$z.err || exit 1; echo phase=$z; python -c "
import json; d=json.load(open('gpurun_out/ph$z.json')); r=d['roofline']; print(round(d['value']), round(d['gpu_stage_pairs_per_s']), round(r['achieved']), round(r['isolated_achieved']))"; done
