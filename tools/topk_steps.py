"""soft top-k per launch vs the fixed step count (B pairs of n x n Sinkhorn outputs, k = 200): separates
the per-step cost from the fixed load / continuation / store cost.   B=32 N=256 python tools/topk_steps.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fpm import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
B, n = int(os.environ.get("B", 32)), int(os.environ.get("N", 256))
s = torch.randn(B, n, n, generator=g) * 0.3
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
ss = ops.sinkhorn(s.to(dev), nn_, nn_, 10, 0.01, True)
k = torch.full((B,), 200.0, device=dev)
steps = torch.empty(B, dtype=torch.int32, device=dev)
out = torch.empty(B, n, n, device=dev)
for it in (0, 2, 4, 10, 20, 40):
    for _ in range(3):
        ops.soft_topk_fwd(ss, nn_, nn_, k, it, 0.01, out=out, steps=steps)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.soft_topk_fwd(ss, nn_, nn_, k, it, 0.01, out=out, steps=steps)
    e1.record()
    torch.cuda.synchronize()
    print("B=%d n=%d iters %2d: %.4f ms per launch, steps %s" % (B, n, it, e0.elapsed_time(e1) / 20,
          sorted(set(steps.tolist()))), flush=True)
