# e2e pairs/s with the host Hungarian pool vs the device LSAP kernel (C3 and C5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in c3 c5; do for m in device host; do
FPM_LSA=$m timeout -k 10 200 python bench.py --config $c --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/lm_${c}_$m.json 2> gpurun_out/lm_${c}_$m.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/lm_${c}_$m.json'));print('$c lsa=$m', round(d['value']), round(d['gpu_stage_pairs_per_s']), round(d['host_lsa_ms_per_step'],1))"
done; done
