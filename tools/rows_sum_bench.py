"""Time fpm_rows_sum (fpm.afau_grad.rows_sum) on training-shaped inputs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fpm  # noqa: E402,F401
from fpm import afau_grad  # noqa: E402

dev = torch.device("cuda", 0)
for R, K in ((16384, 600), (16384, 256), (64, 600), (32, 153600)):
    x = torch.randn(R, K, device=dev)
    ref = x.double().sum(0)
    y = afau_grad.rows_sum(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        afau_grad.rows_sum(x)
    e1.record()
    torch.cuda.synchronize()
    print(R, K, "%.3f ms" % (e0.elapsed_time(e1) / 10), "max err %.2e" % float((y.double() - ref).abs().max()))
