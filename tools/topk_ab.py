"""soft top-k variants (fpm_set_tuning 'topk_fast'): time per launch at B=128, n=256 on bench-like
inputs (Sinkhorn outputs), step counts and max |difference| between the variants."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fpm import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
B, n = int(os.environ.get("B", 128)), int(os.environ.get("N", 256))
s = torch.randn(B, n, n, generator=g) * 0.3
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
ss = ops.sinkhorn(s.to(dev), nn_, nn_, 10, 0.01, True)
k = torch.full((B,), 200.0, device=dev)
res = {}
for fast in (0, 1, 0, 1):
    prev = ops.set_tuning("topk_fast", fast)
    steps = torch.empty(B, dtype=torch.int32, device=dev)
    out = ops.soft_topk_fwd(ss, nn_, nn_, k, 10, 0.01, steps=steps)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.soft_topk_fwd(ss, nn_, nn_, k, 10, 0.01, out=out, steps=steps)
    e1.record()
    torch.cuda.synchronize()
    res[fast] = (out.cpu(), steps.cpu())
    ops.set_tuning("topk_fast", prev)
    print("fast=%d %.4f ms  steps %s" % (fast, e0.elapsed_time(e1) / 10, sorted(set(steps.tolist()))), flush=True)
print("max|diff| %.3g  steps equal %s" % (float((res[1][0] - res[0][0]).abs().max()), torch.equal(res[1][1], res[0][1])))
