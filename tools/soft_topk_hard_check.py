"""Host emulation of the soft_topk mirror's hard output (ops.soft_topk) on the golden soft matrix:
flatten each pair's valid block row-major, stable descending argsort, greedy walk decoded with
the box width -- compared with the reference's own x in tests/golden/soft_topk.npz."""
import os
import sys

import numpy as np
import torch

z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "soft_topk.npz"))
ok = True
for i in range(int(z["ncases"])):
    g = lambda k: z["c%d_%s" % (i, k)]
    ss = torch.from_numpy(g("ss_out"))
    n1, n2, ks, X = g("n1"), g("n2"), g("ks"), g("x")
    B, n1m, n2m = ss.shape
    L = int(n1.max() * n2.max())
    flat = torch.zeros(B, L)
    for b in range(B):
        flat[b, :n1[b] * n2[b]] = ss[b, :n1[b], :n2[b]].reshape(-1)
    top = torch.argsort(flat, dim=-1, descending=True, stable=True)
    x = torch.zeros(B, n1m, n2m)
    for b in range(B):
        m, K = 0, round(float(ks[b]))
        for idx in top[b].tolist():
            if m >= K:
                break
            r, c = idx // n2m, idx % n2m
            if x[b, :, c].sum() < 1 and x[b, r, :].sum() < 1:
                x[b, r, c] = 1
                m += 1
    same = np.array_equal(x.numpy(), X)
    ok &= same
    print(i, same, [int((x[b].numpy() != X[b]).sum()) for b in range(B)], ks, n1, n2)
sys.exit(0 if ok else 1)
