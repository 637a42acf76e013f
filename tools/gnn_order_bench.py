"""GNN layer (C = 17) per launch under graph-2 block orders (fpm_kron_gnn_layer_fwd_ord, a schedule
only): identity, x sweep, Hilbert curve, BFS, random; results checked identical to the identity order.
B pairs of n keypoints (synthetic Delaunay graphs).   B=64 N=512 python tools/gnn_order_bench.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fpm  # noqa: E402
from fpm import ops, synth  # noqa: E402
from fpm.batch import DeviceBatch  # noqa: E402

B, n = int(os.environ.get("B", 64)), int(os.environ.get("N", 512))
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


def hilbert(x, y, order=10):
    d = np.zeros_like(x)
    s = 1 << (order - 1)
    x, y = x.copy(), y.copy()
    while s > 0:
        rx = (x & s) > 0
        ry = (y & s) > 0
        d += s * s * ((3 * rx) ^ ry)
        # rotate
        m = ~ry
        sw = m & rx
        x[sw] = s - 1 - x[sw]
        y[sw] = s - 1 - y[sw]
        t = x[m].copy()
        x[m] = y[m]
        y[m] = t
        s >>= 1
    return d


def bfs(A, start):
    seen = np.zeros(len(A), bool)
    out, q = [], [start]
    seen[start] = True
    while q:
        v = q.pop(0)
        out.append(v)
        for u in np.nonzero(A[v])[0]:
            if not seen[u]:
                seen[u] = True
                q.append(u)
    out += [v for v in range(len(A)) if not seen[v]]
    return np.array(out)


def order(kind, g, rng):
    P = g["P"]
    if kind == "id":
        return np.arange(n)
    if kind == "x":
        return np.argsort(P[:, 0], kind="stable")
    if kind == "hilbert":
        q = (P / np.array([320.0, 240.0]) * 1023).astype(np.int64)
        return np.argsort(hilbert(q[:, 0], q[:, 1]), kind="stable")
    if kind == "bfs":
        return bfs(g["A"], int(np.argmin(P[:, 0])))
    return rng.permutation(n)


rng = np.random.default_rng(0)
res, ref = {}, None
for kind in ("id", "x", "hilbert", "bfs", "rand"):
    o = np.stack([order(kind, p[1], rng) for p in pairs]).astype(np.int32)
    ord2 = torch.as_tensor(o, device=dev)
    args = (X, 17, B, n, n, csr[0], csr[1], bt.n1, bt.n2, wp["gnn1"], Xn, z)
    for _ in range(3):
        ops.gnn_layer(*args, ord2=ord2)
    torch.cuda.synchronize()
    if ref is None:
        ref = (Xn.clone(), z.clone())
    else:
        assert torch.equal(Xn, ref[0]) and torch.equal(z, ref[1]), kind
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.gnn_layer(*args, ord2=ord2)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    print("B=%d n=%d order %-8s median %.3f ms (min %.3f)  outputs identical" % (B, n, kind, sorted(ts)[2], min(ts)),
          flush=True)
