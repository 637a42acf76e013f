# host LSAP paths on the GPU box: micro-bench (1 / 16 threads) and end to end at C3 / C5
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
grep -o "avx512[a-z]*" /proc/cpuinfo | sort -u | tr '\n' ' '; grep -m1 "model name" /proc/cpuinfo
for N in 256 512; do for v in new old; do
  if [ $v = old ]; then export FPM_LSA_DENSE512=1; else unset FPM_LSA_DENSE512; fi
  N=$N timeout -k 10 300 python tools/lsa_bench.py "n=$N $v" 2>&1 | grep threads || exit 1
done; done
for c in c3 c5; do for v in new old new old; do
  if [ $v = old ]; then export FPM_LSA_DENSE512=1; else unset FPM_LSA_DENSE512; fi
  timeout -k 10 200 python bench.py --config $c --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/li_${c}_$v.json 2> gpurun_out/li_${c}_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/li_${c}_$v.json'));print('$c $v', round(d['value']), round(d['gpu_stage_pairs_per_s']), round(d['host_lsa_ms_per_step'],1))"
done; done
