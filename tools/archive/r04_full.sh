#!/bin/bash
# Round 4: full GPU test suite + smoke + default bench (the driver's commands), logs under gpurun_out/.
set -e
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r04b}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
