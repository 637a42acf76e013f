"""Time the Kronecker GNN layer kernel alone on bench-shaped inputs (B pairs, n keypoints)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fpm  # noqa: E402
from fpm import ops, synth  # noqa: E402
from fpm.batch import DeviceBatch  # noqa: E402

B, n = int(os.environ.get("B", 128)), int(os.environ.get("N", 256))
dev = torch.device("cuda", 0)
pairs = synth.make_batch(3, B, n)
bt = DeviceBatch.from_pairs(pairs, dev)
net = fpm.Net(regression=True, backbone=False, dtype="bf16")
wp = net.packed(dev)
plans = [ops.spline_plan(bt.src[s], bt.dst[s], bt.pseudo[s], B * n, n) for s in range(2)]
csr = [ops.plan_csr(plans[s], bt.E[s], B * n) for s in range(2)]
X = torch.randn(B, 17, n, n, device=dev)
Xn = torch.empty_like(X)
z = torch.empty(B, n, n, device=dev)
for C, key in ((17, "gnn1"), (1, "gnn0")):
    for _ in range(3):
        ops.gnn_layer(X, C, B, n, n, csr[0], csr[1], bt.n1, bt.n2, wp[key], Xn, z)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.gnn_layer(X, C, B, n, n, csr[0], csr[1], bt.n1, bt.n2, wp[key], Xn, z)
    e1.record()
    torch.cuda.synchronize()
    print("C=%d dbg=%s %.3f ms" % (C, os.environ.get("FPM_GNN_DBG", "0"), e0.elapsed_time(e1) / 20))
