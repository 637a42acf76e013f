"""Time the L2-streaming Sinkhorn (n > 256) per launch: B pairs of n x n, `iters` steps, tau 0.01,
for each FPM_SK_STREAM_RW given (fpm_set_tuning is not used: the flag is read once per process, so
run one process per value).   python tools/sk_stream_bench.py [B] [n] [iters] [t]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fpm import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
trans = len(sys.argv) > 4 and sys.argv[4] == "t"     # strided view (c along the j axis), as the GNN's
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
s = (torch.randn(B, n, n, generator=g) * 0.3).to(dev)
if trans:
    s = s.transpose(1, 2)
n1 = torch.full((B,), n, dtype=torch.int32, device=dev)
out = torch.empty(B, n, n, device=dev)
if trans:
    out = out.transpose(1, 2)      # the model writes its GNN Sinkhorns through the same strided view
for _ in range(3):
    ops.sinkhorn(s, n1, n1, iters, 0.01, True, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
R = 10
for _ in range(R):
    ops.sinkhorn(s, n1, n1, iters, 0.01, True, out=out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / R
print("RW=%s B=%d n=%d iters=%d%s: %.3f ms per launch, %.1f us per half-step, %.0f GB/s of s re-reads" % (
    os.environ.get("FPM_SK_STREAM_RW", "4"), B, n, iters, " transposed" if trans else "", ms, ms * 1e3 / iters, B * n * n * 4 * iters / ms / 1e6))
