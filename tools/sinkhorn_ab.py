"""Sinkhorn forward variants (fpm_set_tuning 'sinkhorn_fast': 0 log, 1 shifted lse, 2 = 1 with scalar stream loads): time per launch at B=128, n=256,
20 iterations, and max |difference| between the variants and against a float64 restatement."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fpm import ops  # noqa: E402
import oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
cases = ((128, 256, 20, False), (64, 256, 10, True), (128, 128, 20, False), (128, 512, 20, False),
         (64, 512, 10, True))
for B, n, iters, ragged in cases[int(os.environ.get("FIRST", 0)):]:
    s = torch.randn(B, n, n, generator=g) * 0.3
    n1 = torch.full((B,), n, dtype=torch.int32)
    n2 = n1.clone()
    if ragged:
        n1[::2] = n - 37
        n2[1::3] = n - 50
    sd, n1d, n2d = s.to(dev), n1.to(dev), n2.to(dev)
    outs = {}
    for fast in (0, 1, 2):
        prev = ops.set_tuning("sinkhorn_fast", fast)
        out = ops.sinkhorn(sd, n1d, n2d, iters, 0.01, True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.sinkhorn(sd, n1d, n2d, iters, 0.01, True, out=out)
        e1.record()
        torch.cuda.synchronize()
        outs[fast] = out.cpu()
        ops.set_tuning("sinkhorn_fast", prev)
        print("B=%d n=%d iters=%d ragged=%s fast=%d %.4f ms" % (B, n, iters, ragged, fast, e0.elapsed_time(e1) / 10))
    ref = O.pygm_sinkhorn(s[:4].double(), n1[:4].tolist(), n2[:4].tolist(), dummy_row=True, max_iter=iters, tau=0.01)
    print("   max|1-0| %.3g  max|2-1| %.3g   vs f64: 0 %.3g 1 %.3g 2 %.3g" % (
        float((outs[1] - outs[0]).abs().max()), float((outs[2] - outs[1]).abs().max()),
        float((outs[0][:4].double() - ref).abs().max()), float((outs[1][:4].double() - ref).abs().max()),
        float((outs[2][:4].double() - ref).abs().max())))
