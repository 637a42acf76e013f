"""Diagnostic: SplineConv product rows (y workspace) with the persistent product GEMM vs the one-shot
phase kernel on one side of a synthetic batch; prints where they differ."""
import ctypes
import sys

import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import fpm
from fpm import ops, params, synth
from fpm.batch import DeviceBatch
from fpm import config as C

DEV = torch.device("cuda", 0)
npairs, n = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (3, 64)
sd = params.init_params(7)
net = fpm.Net(regression=True, backbone=False, dtype="bf16")
net.load_state_dict(sd)
wp = net.packed(DEV)
bt = DeviceBatch.from_pairs(synth.make_batch(17, npairs, n), DEV)
side = 0
nn_ = bt.B * bt.nmax[side]
E = bt.E[side]
plan = ops.spline_plan(bt.src[side], bt.dst[side], bt.pseudo[side], nn_, bt.nmax[side], bt.max_graph_edges(side))
x_op = ops.cast_bf16(bt.x[side])
arows, cell_off = ops.spline_plan_rows(plan, E, nn_)
base = plan.data_ptr()
off = cell_off.cpu().tolist()
extra = plan[(cell_off.data_ptr() - base):(cell_off.data_ptr() - base) + 4 * 29].view(torch.int32).cpu().tolist()
rows = off[26]
print("rows", rows, "cell_off", off, "tile counts (128, 256):", extra[27:29])
ys = []
for v in (0, 1):
    prev = ops.set_tuning("gemm_persist", v)
    yws = ops.spline_y_ws(ops.BF16, E, nn_, DEV)
    yws.fill_(0x55)
    h = torch.empty(nn_, C.NODE_FEATURE_DIM, device=DEV, dtype=torch.bfloat16)
    ops.spline_conv(x_op, plan, E, nn_, bt.nmax[side], bt.n[side], wp["W0"], wp["bias0"], yws, 0, out_t=h)
    torch.cuda.synchronize()
    ops.set_tuning("gemm_persist", prev)
    ys.append(yws[:rows * 768 * 2].view(torch.int16).view(rows, 768).clone())
d = ys[0] != ys[1]
print("mismatching elements", int(d.sum()), "of", d.numel())
if d.any():
    r, c = torch.nonzero(d, as_tuple=True)
    rr, cc = r.cpu(), c.cpu()
    print("rows (first 20):", sorted(set(rr.tolist()))[:20])
    print("cols mod 256 hist (by 16):", torch.bincount((cc % 256) // 16, minlength=16).tolist())
    print("row mod 256 hist (by 16):", torch.bincount((rr % 256) // 16, minlength=16).tolist())
    print("col tiles:", torch.bincount(cc // 256, minlength=3).tolist())
    grp = [next(k for k in range(26) if off[k] <= x < off[k + 1]) for x in rr[:2000].tolist()]
    print("groups:", sorted(set(grp)))
    k = 0
    print("sample", int(rr[k]), int(cc[k]), int(ys[0][rr[k], cc[k]]), int(ys[1][rr[k], cc[k]]))
if d.any():
    y1 = ys[1]
    r0, c0 = int(rr[0]), int(cc[0])
    row = y1[r0].cpu()
    ref = ys[0][r0].cpu()
    lo = c0 - c0 % 256
    print("row", r0, "persist cols", lo + 88, ":", row[lo + 88:lo + 136].tolist())
    print("row", r0, "oneshot cols", lo + 88, ":", ref[lo + 88:lo + 136].tolist())
    wrong_rows = sorted(set(rr.tolist()))
    print("n wrong rows", len(wrong_rows), "per-row wrong col count (first 10):",
          [int(d[x].sum()) for x in wrong_rows[:10]])
    a = arows[:rows].cpu()
    print("arows around row:", a[max(0, r0 - 40):r0 + 40].tolist())
