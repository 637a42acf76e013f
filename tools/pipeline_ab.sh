# end-to-end pairs/s vs pipeline shape: tail halvings (FPM_TAIL) and chunk count (FPM_CHUNKS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in c3 c5; do for cfg in "1 8" "2 8" "1 6" "2 6" "1 8" "2 8"; do
  set -- $cfg
  FPM_TAIL=$1 FPM_CHUNKS=$2 timeout -k 10 200 python bench.py --config $c --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/pl_${c}.json 2> gpurun_out/pl_${c}.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/pl_${c}.json'));print('$c tail=$1 chunks=$2', round(d['value']), round(d['gpu_stage_pairs_per_s']), round(d['host_lsa_ms_per_step'],1), round(d['ms_per_step'],2))"
done; done
