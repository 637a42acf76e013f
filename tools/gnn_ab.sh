set -o pipefail
cd "$GRAFT_REPO_ROOT"
for u in 1 2 3 1 2 3; do FPM_GNN_UNROLL=$u timeout -k 10 120 python tools/gnn_bench.py 2>&1 | tail -2 | sed "s/^/U=$u /"; done
