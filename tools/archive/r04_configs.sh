#!/bin/bash
# the non-headline SURVEY §8 configs on the current tree, each with its cpu_baseline and self-check
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in c2 c4 c5; do
  timeout -k 10 500 python bench.py --config $c > gpurun_out/r04x_bench_$c.json 2> gpurun_out/r04x_bench_$c.err || { tail -20 gpurun_out/r04x_bench_$c.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r04x_bench_$c.json').read().strip().splitlines()[-1])
print('$c', d['metric'], round(d['value']), d['unit'], 'selfcheck', d.get('timed_batch_selfcheck'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
