"""Sinkhorn forward kernel alone, per variant (fpm_set_tuning "sinkhorn_lform"): B pairs of n x n,
20 steps, tau 0.05 (the GNN's Sinkhorn), HIP events around 20 launches.
    python tools/sk_bench.py [B] [n]"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fpm import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
s = (torch.randn(B, n, n, generator=g) * 0.3).to(dev)
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
out = torch.empty_like(s)
res = {}
for v in (0, 1):
    prev = ops.set_tuning("sinkhorn_lform", v)
    for _ in range(3):
        ops.sinkhorn(s, nn_, nn_, 20, 0.05, True, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.sinkhorn(s, nn_, nn_, 20, 0.05, True, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    ops.set_tuning("sinkhorn_lform", prev)
    steps = B * 20 * n * n
    res[v] = ms
    print("lform=%d  %.3f ms per launch  %.2f G entry-steps/s" % (v, ms, steps / ms / 1e6))
print("lform 1 vs 0: %.2fx" % (res[0] / res[1]))
