# end-to-end pairs/s vs host LSA pool size (FPM_LSA_THREADS) at C3 / C5
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in c3 c5; do for t in 16 32 24 16 32; do
  FPM_LSA_THREADS=$t timeout -k 10 200 python bench.py --config $c --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/th_${c}_$t.json 2> gpurun_out/th_${c}_$t.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/th_${c}_$t.json'));print('$c threads=$t', round(d['value']), round(d['gpu_stage_pairs_per_s']), round(d['host_lsa_ms_per_step'],1), d['ms_per_step'])"
done; done
