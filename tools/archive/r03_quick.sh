#!/bin/bash
# round-3 quick GPU check: selected tests (pytest -k expression in $1, optional), then the default bench
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${TAG:-r03}
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$1" > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/${tag}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 500 python bench.py --steps 5 --warmup 1 --cpu-pairs 8 ${BENCH_ARGS} > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
  cat gpurun_out/${tag}_bench.json; grep "step:" gpurun_out/${tag}_bench.err | tail -6
fi
