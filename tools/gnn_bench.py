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
X1 = X[:, :1].contiguous()
Xn = torch.empty_like(X)
z = torch.empty(B, n, n, device=dev)
variants = [tuple((k, int(v)) for k, v in (kv.split("=") for kv in a.split(","))) for a in sys.argv[1:]] or [()]
ROUNDS = int(os.environ.get("ROUNDS", 5))


ORD = {}


def time_layer(C, key, Xc, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.gnn_layer(Xc, C, B, n, n, csr[0], csr[1], bt.n1, bt.n2, wp[key], Xn, z)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
for rnd in range(ROUNDS):                 # variants interleaved, median over rounds
    for var in variants:
        prev = [(k, ops.set_tuning(k, v)) for k, v in var]
        for C, key in ((17, "gnn1"), (1, "gnn0")):
            Xc = X if C == 17 else X1
            ops.gnn_layer(Xc, C, B, n, n, csr[0], csr[1], bt.n1, bt.n2, wp[key], Xn, z)
            torch.cuda.synchronize()
            res.setdefault((var, C), []).append(time_layer(C, key, Xc))
        for k, v in prev:
            ops.set_tuning(k, v)
for (var, C), ts in res.items():
    ms = sorted(ts)[len(ts) // 2]
    gb = B * n * n * 4 * (C + 17) / 1e9        # algorithmic: X in (C channels) + 16 channels + z out
    print("%-40s C=%-2d median %.3f ms (min %.3f)  %.0f GB/s algorithmic" % (var, C, ms, min(ts), gb / (ms / 1e3)))

# phase split (timing only): graph-2 and/or graph-1 neighbour lists emptied (ptr all zero)
if os.environ.get("GNN_PHASES"):
    zp = torch.zeros(B * n + 1, device=dev, dtype=torch.int32)
    zcsr = (zp.data_ptr(), zp.data_ptr())
    for tag, c1, c2 in (("full", csr[0], csr[1]), ("no-g2-agg", csr[0], zcsr), ("no-g1-agg", zcsr, csr[1]),
                        ("mlp-only", zcsr, zcsr)):
        for _ in range(3):
            ops.gnn_layer(X, 17, B, n, n, c1, c2, bt.n1, bt.n2, wp["gnn1"], Xn, z)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.gnn_layer(X, 17, B, n, n, c1, c2, bt.n1, bt.n2, wp["gnn1"], Xn, z)
        e1.record()
        torch.cuda.synchronize()
        print("phase %-10s C=17 %.3f ms" % (tag, e0.elapsed_time(e1) / 20))
