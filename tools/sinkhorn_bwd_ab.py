"""Sinkhorn backward kernels (fpm_set_tuning 'sinkhorn_bwd_reg': 1 register tile with the forward
replay, 0 general): time per launch and max relative difference, at the training shapes
(B = 64 pairs, n = 256; GNN Sinkhorn 20 steps, final 10 steps, tau 0.05)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fpm import ops, train  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
for B, n, iters, tau in ((64, 256, 20, 0.05), (64, 256, 10, 0.05), (128, 128, 20, 0.05)):
    s = (torch.randn(B, n, n, generator=g) * 0.3).to(dev)
    dp = torch.randn(B, n, n, generator=g).to(dev)
    n1 = torch.full((B,), n, dtype=torch.int32, device=dev)
    outs = {}
    for reg in (1, 0):
        prev = ops.set_tuning("sinkhorn_bwd_reg", reg)
        ds = train.sinkhorn_bwd(s, dp, n1, n1, iters, tau, True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ds = train.sinkhorn_bwd(s, dp, n1, n1, iters, tau, True)
        e1.record()
        torch.cuda.synchronize()
        ops.set_tuning("sinkhorn_bwd_reg", prev)
        outs[reg] = ds.float().cpu()
        print("B=%d n=%d iters=%d reg=%d  %.3f ms" % (B, n, iters, reg, e0.elapsed_time(e1) / 5))
    d = (outs[1] - outs[0]).abs().max() / outs[0].abs().max()
    print("   max rel |reg - general| %.3g" % float(d))
