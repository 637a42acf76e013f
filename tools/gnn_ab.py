"""A/B of the GNN-layer kernel variants (fpm_set_tuning 'gnn_group' / 'gnn_unroll'): time per
launch at B=128, n=256 and bit-equality of the outputs against the default variant."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fpm  # noqa: E402
from fpm import ops, synth  # noqa: E402
from fpm.batch import DeviceBatch  # noqa: E402

B, n = int(os.environ.get("B", 128)), int(os.environ.get("N", 256))
dev = torch.device("cuda", 0)
bt = DeviceBatch.from_pairs(synth.make_batch(3, B, n), dev)
wp = fpm.Net(regression=True, backbone=False, dtype="bf16").packed(dev)
plans = [ops.spline_plan(bt.src[s], bt.dst[s], bt.pseudo[s], B * n, n) for s in range(2)]
csr = [ops.plan_csr(plans[s], bt.E[s], B * n) for s in range(2)]
C = int(os.environ.get("C", 17))
X = torch.randn(B, C, n, n, device=dev)
key_w = "gnn1" if C == 17 else "gnn0"
ref = None
for key, val in [(k, int(v)) for k, v in (a.split("=") for a in sys.argv[1:])]:
    prev = ops.set_tuning(key, val)
    Xn = torch.zeros(B, 17, n, n, device=dev)
    z = torch.zeros(B, n, n, device=dev)
    for _ in range(3):
        ops.gnn_layer(X, C, B, n, n, csr[0], csr[1], bt.n1, bt.n2, wp[key_w], Xn, z)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.gnn_layer(X, C, B, n, n, csr[0], csr[1], bt.n1, bt.n2, wp[key_w], Xn, z)
    e1.record()
    torch.cuda.synchronize()
    out = (Xn[:, :16].clone(), z.clone())
    if ref is None:
        ref = out
    same = torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
    print("%s=%d %.3f ms  identical=%s" % (key, val, e0.elapsed_time(e1) / 20, same), flush=True)
    ops.set_tuning(key, prev)
