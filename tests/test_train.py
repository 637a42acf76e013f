"""Training backward: the HIP vector-Jacobian products against autograd
through the CPU oracle on identical inputs.

Per-op tests use a float64 oracle (the reference of the gradient), the end-to-end step uses the
fp32 oracle (so both sides take the same soft top-k step count and the same Hungarian matches).
Gradients are compared relative to their own scale: err = max|g - g_ref| / max|g_ref|.  The
tolerances are written per test; the tau = 0.01 Sinkhorns amplify fp32 forward differences,
so the end-to-end bound is looser than the per-op ones.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F_

import fpm
from fpm import ops, params, synth, train
from fpm.batch import DeviceBatch
import oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _i32(x):
    return torch.as_tensor(np.asarray(x), dtype=torch.int32, device=DEV)


def _rel(a, b, floor=1e-12):
    """max|a - b| / max(max|b|, floor).  ``floor``: the scale of a gradient that is analytically
    zero (e.g. a bias feeding a Sinkhorn, which is shift-invariant) is that of its neighbours."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp(min=floor))


@pytest.fixture(scope="module")
def sd():
    return params.init_params(7)


# ------------------------------------------------------------------------------------- Sinkhorn
@pytest.mark.parametrize("reg", [1, 0])
@pytest.mark.parametrize("n1s,n2s,iters,tau", [
    ((8, 8), (8, 8), 10, 0.05),
    ((32, 20, 32), (32, 32, 17), 20, 0.01),          # dummy rows + transposed pair
    ((64, 50), (64, 64), 10, 0.01),
    ((128,), (128,), 20, 0.01),
    ((256, 200, 131), (256, 256, 240), 21, 0.02),    # register tile 8x8, odd steps, both dummy sides
    ((90, 256), (256, 77), 1, 0.05),                 # a single step
])
def test_sinkhorn_bwd_vs_autograd(reg, n1s, n2s, iters, tau):
    """Both backward kernels (register tile with the forward's replay, n <= 256; general) against
    autograd through the float64 oracle, for contiguous and transposed-storage inputs."""
    g = torch.Generator().manual_seed(sum(n1s) + iters)
    B = len(n1s)
    n1max, n2max = max(n1s), max(n2s)
    s = torch.randn(B, n1max, n2max, generator=g, dtype=torch.float64) * 0.05
    dp = torch.randn(B, n1max, n2max, generator=g, dtype=torch.float64)
    sl = s.clone().requires_grad_(True)
    out = O.pygm_sinkhorn(sl, n1s, n2s, dummy_row=True, max_iter=iters, tau=tau)
    (out * dp).sum().backward()
    ref = sl.grad
    sd_ = s.float().to(DEV)
    prev = ops.set_tuning("sinkhorn_bwd_reg", reg)
    try:
        ds = train.sinkhorn_bwd(sd_, dp.float().to(DEV), _i32(n1s), _i32(n2s), iters, tau, True)
        # strided (transposed-storage) input view: the same gradient (bit-identical for the general
        # kernel, which walks algorithmic coordinates; the register tile reduces along the storage
        # axes, so rounding may differ)
        sT = sd_.transpose(1, 2).contiguous().transpose(1, 2)
        ds2 = train.sinkhorn_bwd(sT, dp.float().to(DEV), _i32(n1s), _i32(n2s), iters, tau, True)
    finally:
        ops.set_tuning("sinkhorn_bwd_reg", prev)
    assert _rel(ds, ref) < 2e-4
    if reg:
        assert _rel(ds2, ref) < 2e-4 and _rel(ds2, ds.double().cpu()) < 1e-5
    else:
        assert torch.equal(ds.cpu(), ds2.cpu())
    # padding of the box stays zero
    for b in range(B):
        assert ds[b, n1s[b]:].abs().sum() == 0 and ds[b, :, n2s[b]:].abs().sum() == 0


# ----------------------------------------------------------------------------------- soft top-k
@pytest.mark.parametrize("n1s,n2s,kf", [
    ((16,), (16,), 0.5),
    ((32, 24), (32, 30), 0.8),
    ((64,), (64,), 0.3),
])
def test_soft_topk_bwd_vs_autograd(n1s, n2s, kf):
    g = torch.Generator().manual_seed(sum(n1s))
    B = len(n1s)
    n1max, n2max = max(n1s), max(n2s)
    ss = torch.rand(B, n1max, n2max, generator=g, dtype=torch.float64)
    k = torch.tensor([round(kf * min(a, b)) for a, b in zip(n1s, n2s)], dtype=torch.float64)
    dd = torch.randn(B, n1max, n2max, generator=g, dtype=torch.float64)
    # fp32 values on both sides so the forwards take the same number of steps
    ss32 = ss.float()
    sl = ss32.double().clone().requires_grad_(True)
    out = O.soft_topk(sl, k, n1s, n2s, 10, 0.01)
    (out * dd).sum().backward()
    steps = torch.empty(B, dtype=torch.int32, device=DEV)
    ops.soft_topk_fwd(ss32.to(DEV), _i32(n1s), _i32(n2s), k.float().to(DEV), 10, 0.01, steps=steps)
    dss = ops.soft_topk_bwd(ss32.to(DEV), _i32(n1s), _i32(n2s), k.float().to(DEV), steps, 0.01, dd.float().to(DEV))
    assert _rel(dss, sl.grad) < 1e-3


def test_soft_topk_bwd_tied_anchors():
    """Several entries equal to the min and the max: the anchors' gradient is split evenly over
    the ties (torch min()/max() backward)."""
    n = 12
    ss = torch.rand(1, n, n, generator=torch.Generator().manual_seed(3)).double()
    ss[0, 0, :3] = ss.min()
    ss[0, 5, 2:4] = ss.max()
    k = torch.tensor([6.0], dtype=torch.float64)
    dd = torch.randn(1, n, n, generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    sl = ss.float().double().clone().requires_grad_(True)
    (O.soft_topk(sl, k, [n], [n], 10, 0.01) * dd).sum().backward()
    steps = torch.empty(1, dtype=torch.int32, device=DEV)
    ops.soft_topk_fwd(ss.float().to(DEV), _i32([n]), _i32([n]), k.float().to(DEV), 10, 0.01, steps=steps)
    dss = ops.soft_topk_bwd(ss.float().to(DEV), _i32([n]), _i32([n]), k.float().to(DEV), steps, 0.01,
                            dd.float().to(DEV))
    assert _rel(dss, sl.grad) < 1e-3


# ------------------------------------------------------------------------ Kronecker aggregation
def test_kron_agg_forward_and_adjoint():
    n1s, n2s = [30, 24, 17], [28, 30, 20]
    B, nm = 3, 30
    pairs = synth.make_batch(5, B, n1s, n2s)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    sides = [train._Side(bt, 0), train._Side(bt, 1)]
    g = torch.Generator().manual_seed(1)
    for C in (1, 17):
        X = torch.randn(B, C, nm, nm, generator=g)
        Y = torch.randn(B, C, nm, nm, generator=g)
        AX = torch.empty(B, C, nm, nm, device=DEV)
        ATY = torch.empty(B, C, nm, nm, device=DEV)
        ops.kron_agg(X.to(DEV), C, B, nm, nm, sides[0].csr, sides[1].csr, sides[0].csr[0], sides[1].csr[0],
                     bt.n1, bt.n2, False, AX)
        ops.kron_agg(Y.to(DEV), C, B, nm, nm, sides[0].out_csr(), sides[1].out_csr(), sides[0].csr[0],
                     sides[1].csr[0], bt.n1, bt.n2, True, ATY)
        AX, ATY = AX.cpu(), ATY.cpu()
        for b in range(B):
            ei1 = torch.as_tensor(pairs[b][0]["edge_index"])
            ei2 = torch.as_tensor(pairs[b][1]["edge_index"])
            x = X[b].reshape(C, nm * nm).t()
            ref = O.pattern_mean_factorized(x, ei1, ei2, nm, nm, n1s[b], n2s[b])
            assert (AX[b].reshape(C, -1).t() - ref).abs().max() < 1e-5
        lhs = float((AX.double() * Y.double()).sum())
        rhs = float((X.double() * ATY.double()).sum())
        assert abs(lhs - rhs) < 1e-4 * max(1.0, abs(lhs))


# ---------------------------------------------------------------------------------- SplineConv
@pytest.mark.parametrize("scatter", ["1", "0"])
def test_spline_layers_bwd_vs_autograd(sd, scatter, monkeypatch):
    """Both SplineConv backward forms (atomic-free scatter over out-edges with the forward's argmax
    slots; atomic combine backward) against autograd through the float64 oracle."""
    monkeypatch.setenv("FPM_SPLINE_SCATTER", scatter)
    n1s = [40, 33, 21]
    pairs = synth.make_batch(11, 3, n1s, n2=[40, 33, 21])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    side = train._Side(bt, 0)
    nm = bt.nmax[0]
    pre = params.SPLINE_PREFIX
    W = {k: sd[k].clone().to(DEV).requires_grad_(True) for k in sd if k.startswith(pre) and sd[k].is_floating_point()}
    x0 = bt.x[0].clone().requires_grad_(True)
    h = train.SplineLayerFn.apply(x0, W[pre + ".0.weight"], W[pre + ".0.root"], W[pre + ".0.bias"], None, side, 0, "f32")
    o = train.SplineLayerFn.apply(h, W[pre + ".1.weight"], W[pre + ".1.root"], W[pre + ".1.bias"], x0, side, 1, "f32")
    R = torch.randn(o.shape, generator=torch.Generator().manual_seed(2)).to(DEV)
    (o * R).sum().backward()
    # oracle (float64) per graph, the same upstream gradient on the valid rows
    Wr = {k: sd[k].double().clone().requires_grad_(True) for k in W}
    sdd = dict(sd)
    sdd.update(Wr)
    gx = []
    Rc = R.cpu().double()
    tot = None
    for b in range(bt.B):
        gph = pairs[b][0]
        xb = torch.from_numpy(gph["x"]).double().requires_grad_(True)
        ref = O.siamese_sconv(xb, torch.from_numpy(gph["edge_index"]), torch.from_numpy(gph["pseudo"]), sdd)
        term = (ref * Rc[b * nm:b * nm + gph["n"]]).sum()
        tot = term if tot is None else tot + term
        gx.append(xb)
    tot.backward()
    for b in range(bt.B):
        n = pairs[b][0]["n"]
        assert _rel(x0.grad[b * nm:b * nm + n], gx[b].grad) < 1e-4
    for k in W:
        assert _rel(W[k].grad, Wr[k].grad) < 1e-4, k


# ---------------------------------------------------------------------------------------- GNN
@pytest.mark.parametrize("C,layer", [(1, 0), (17, 1)])
def test_gnn_layer_bwd_vs_autograd(sd, C, layer):
    n1s, n2s = [24, 20], [24, 22]
    B, nm = 2, 24
    pairs = synth.make_batch(13, B, n1s, n2s)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    g = train._GnnCtx(bt, train._Side(bt, 0), train._Side(bt, 1))
    pre = "gnn_layer_%d." % layer
    names = ["conv2.lin_l.weight", "conv2.lin_l.bias", "conv2.lin_r.weight", "n_self_func.0.weight",
             "n_self_func.0.bias", "n_self_func.2.weight", "n_self_func.2.bias", "classifier.weight",
             "classifier.bias"]
    Pg = [sd[pre + k].clone().to(DEV).requires_grad_(True) for k in names]
    gen = torch.Generator().manual_seed(C + layer)
    X = (torch.randn(B, C, nm, nm, generator=gen) * 0.5)
    Xg = X.clone().to(DEV).requires_grad_(True)
    Xn = train.GnnLayerFn.apply(Xg, *Pg, g)
    R = torch.randn(B, 17, nm, nm, generator=gen)
    (Xn * R.to(DEV)).sum().backward()
    Pr = {pre + k: sd[pre + k].double().clone().requires_grad_(True) for k in names}
    sdd = dict(sd)
    sdd.update(Pr)
    tot = None
    xs = []
    for b in range(B):
        ei1 = torch.as_tensor(pairs[b][0]["edge_index"])
        ei2 = torch.as_tensor(pairs[b][1]["edge_index"])
        x = X[b].double().reshape(C, nm * nm).t().clone().requires_grad_(True)
        agg_fn = lambda t, ei1=ei1, ei2=ei2, b=b: O.pattern_mean_factorized(t, ei1, ei2, nm, nm, n1s[b], n2s[b])
        out = O.gnn_layer(x, sdd, layer, agg_fn, nm, nm, n1s[b], n2s[b])
        term = (out * R[b].double().reshape(17, -1).t()).sum()
        tot = term if tot is None else tot + term
        xs.append(x)
    tot.backward()
    for b in range(B):
        assert _rel(Xg.grad[b].reshape(C, -1).t(), xs[b].grad) < 2e-4
    scale = max(float(Pr[pre + k].grad.abs().max()) for k in names)
    for k, p in zip(names, Pg):
        assert _rel(p.grad, Pr[pre + k].grad, 1e-2 * scale) < 2e-4, k




# ------------------------------------------------------------ AFA-U reference at device intermediates
def afau_grads_anchored(sv, P, dks, names):
    """fp64 autograd of the AFA-U regressor's parameter gradients (afau.py:54-300, ngm.py:386-412)
    evaluated stage by stage AT THE DEVICE FORWARD'S OWN SAVED INTERMEDIATES (``fpm.afau_grad``'s
    AfauSaved): the gradient jumps at the FFN ReLU kinks and at the max pool, so a reference that
    recomputes those decisions in another precision can land on other branches than the device for
    values within an ulp of a kink (round 3: a 1-ulp change of ss moved the end-to-end check from
    <2e-3 to 5.3e-3).  Here the FFN ReLU masks are the device's (h > 0); the mixed-score MLP's kinks
    are decided exactly either way (its pre-activation c w1 + b1 is one fma, exact in fp64); the max
    pool and the head take their decisions from the device's tail inputs (o1 + ff).  Every stage's
    arithmetic is fp64 autograd of the reference statement.  -> {name: grad (fp64, CPU)}."""
    dd = torch.float64
    pre = "encoder_k.layers.0."
    L = {k: P(k).detach().to(dd).clone().requires_grad_(True) for k in names}
    g = lambda blk, k: L[pre + blk + "_encoding_block." + k]
    inorm = lambda x, w, b, nb, Pn: F_.instance_norm(x.view(nb, Pn, -1).transpose(1, 2), weight=w, bias=b,
                                                     eps=1e-5).transpose(1, 2).reshape(nb * Pn, -1)
    dks = dks.to(dd)
    # 1) tails: y = IN2(o1 + ff) per block, max over positions, heads, ks
    leaf = {}
    gm = {}
    for blk in ("row", "col"):
        st = sv.blk[blk]
        nb, Pn = st["nb"], st["P"]
        o1 = st["o1"].to(dd).clone().requires_grad_(True)
        ff = st["ff"].to(dd).clone().requires_grad_(True)
        leaf[blk] = (o1, ff)
        y = inorm(o1 + ff, g(blk, "add_n_normalization_2.norm.weight"), g(blk, "add_n_normalization_2.norm.bias"),
                  nb, Pn)
        gm[blk] = y.view(nb, Pn, -1).max(dim=1).values
    gr, gc = gm["row"], gm["col"][sv.inv.long()]
    head = lambda x, h: F_.linear(F_.relu(F_.linear(x, L[h + ".0.weight"], L[h + ".0.bias"])), L[h + ".2.weight"],
                                  L[h + ".2.bias"]).squeeze(-1)
    ks = torch.sigmoid((head(gr, "final_row") + head(gc, "final_col")) / 2)
    (ks * dks).sum().backward()
    for blk in ("row", "col"):
        st = sv.blk[blk]
        nb, Pn = st["nb"], st["P"]
        o1t, fft = leaf[blk]
        # 2) FFN with the device's ReLU decisions: ff = W2 (mask o (W1 o1 + b1)) + b2
        o1 = st["o1"].to(dd).clone().requires_grad_(True)
        mask = (st["h"] > 0).to(dd)
        ff = F_.linear(mask * F_.linear(o1, g(blk, "feed_forward.W1.weight"), g(blk, "feed_forward.W1.bias")),
                       g(blk, "feed_forward.W2.weight"), g(blk, "feed_forward.W2.bias"))
        ff.backward(fft.grad)
        do1 = o1t.grad + o1.grad
        # 3) first instance norm: row input = combine(att), col input = one-hot + combine bias
        w1n, b1n = g(blk, "add_n_normalization_1.norm.weight"), g(blk, "add_n_normalization_1.norm.bias")
        if blk == "row":
            mh = sv.mh.to(dd).clone().requires_grad_(True)
            inorm(mh, w1n, b1n, nb, Pn).backward(do1)
            # 4) combine: mh = att Wc^T + bc
            att = sv.att.to(dd).clone().requires_grad_(True)
            F_.linear(att, g(blk, "multi_head_combine.weight"), g(blk, "multi_head_combine.bias")).backward(mh.grad)
            # 5) cross-set attention from ss (R0 = 0: q = 0, the dot-product input is 0; afau.py:231-300)
            B, n1max, n2max = sv.B, sv.n1max, sv.n2max
            cost = sv.ss.to(dd)
            w1, b1 = g(blk, "mixed_score_MHA.mix1_weight"), g(blk, "mixed_score_MHA.mix1_bias")
            w2, b2 = g(blk, "mixed_score_MHA.mix2_weight"), g(blk, "mixed_score_MHA.mix2_bias")
            two = torch.stack((torch.zeros(B, 16, n1max, n2max, dtype=dd, device=cost.device),
                               cost[:, None].expand(B, 16, n1max, n2max)), dim=4).transpose(1, 2)
            ms1 = torch.matmul(two, w1) + b1[None, None, :, None, :]
            mixed = (torch.matmul(F_.relu(ms1), w2) + b2[None, None, :, None, :]).transpose(1, 2).squeeze(4)
            a = torch.softmax(mixed, dim=3)                                   # (B, H, n1max, n2max)
            Wv = g(blk, "Wv.weight")                                          # (256, 600)
            colmask = (torch.arange(n2max, device=cost.device)[None, :] < sv.n2.long()[:, None]).to(dd)
            v = Wv[:, :n2max].t()[None] * colmask[:, :, None]                 # one-hot col rows -> Wv columns
            v = v.view(B, n2max, 16, 16).transpose(1, 2)
            out = torch.matmul(a, v).transpose(1, 2).reshape(B * n1max, 256)
            out.backward(att.grad)
        else:
            n2u = sv.n2u.long()
            idx = torch.arange(Pn, device=n2u.device)
            x = ((idx[None, :, None] == torch.arange(600, device=n2u.device)[None, None, :])
                 & (idx[None, :, None] < n2u.view(-1, 1, 1))).to(dd).view(nb * Pn, 600)
            inorm(x + g(blk, "multi_head_combine.bias"), w1n, b1n, nb, Pn).backward(do1)
    return {k: (v.grad.detach().cpu() if v.grad is not None else None) for k, v in L.items()}

# ------------------------------------------------------------------------------- whole step
def _gt(pairs):
    B = len(pairs)
    n1 = [p[0]["n"] for p in pairs]
    n2 = [p[1]["n"] for p in pairs]
    gt = torch.zeros(B, max(n1), max(n2))
    for b in range(B):
        m = min(n1[b], n2[b])
        gt[b, torch.arange(m), torch.arange(m)] = 1.0
    return gt, n1, n2


def _train_step_compare(pairs, sd, labels):
    gt, n1, n2 = _gt(pairs)
    net = fpm.Net(regression=True, backbone=False, dtype="f32")
    net.load_state_dict(sd)
    net.to(DEV).train()
    bt = DeviceBatch.from_pairs(pairs, DEV)
    from fpm import afau_grad
    captured = []
    real_fwd = afau_grad.forward

    def spy(P, ss, bt_, **kw):         # keep the device AFA-U forward's saved intermediates
        ks_, sv_ = real_fwd(P, ss, bt_, **kw)
        captured.append((ks_.detach().clone(), sv_))
        return ks_, sv_
    afau_grad.forward = spy
    try:
        out = net({"fpm_batch": bt, "gt_perm_mat": gt, "label": labels})
        loss = train.permutation_loss(out["ds_mat"], gt, n1, n2) + out["ks_loss"] + out["cls_loss"]
        loss.backward()
    finally:
        afau_grad.forward = real_fwd
    sdl = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running_" not in k else v.clone())
           for k, v in sd.items()}
    ref = O.forward(pairs, sdl, regression=True, training=True, gt_perm=gt, labels=labels)
    rl = O.permutation_loss(ref["ds_mat"], gt, n1, n2) + ref["ks_loss"] + ref["cls_loss"]
    rl.backward()
    assert torch.equal(out["perm_mat"].cpu(), ref["perm_mat"])
    assert abs(float(loss) - float(rl)) < 1e-4 * max(1.0, abs(float(rl)))
    errs = {}
    pd = dict(net.named_parameters())
    group = lambda k: k.split(".")[0]
    scale = {}
    for k, v in sdl.items():
        if v.is_floating_point() and v.requires_grad and v.grad is not None:
            scale[group(k)] = max(scale.get(group(k), 0.0), float(v.grad.abs().max()))
    for k, v in sdl.items():
        if not (v.is_floating_point() and v.requires_grad):
            continue
        gr = pd[k].grad
        if v.grad is None:
            assert gr is None or float(gr.abs().max()) == 0.0, k
            continue
        assert gr is not None, k
        errs[k] = _rel(gr, v.grad, 1e-3 * scale[group(k)])
        if k.endswith(ZERO_GRAD) and not k.startswith("classifier"):
            assert float(gr.abs().max()) < 1e-3 * scale[group(k)], k
    # AFA-U: its gradient is discontinuous (ReLU kinks of the FFN and the +-10 mixed-score MLP, the
    # max pool) and, through the softmax backward, a sum with heavy cancellation, so a reference that
    # re-derives the forward (oracle, or any replay in another precision) can take other branches for
    # values within an ulp of a kink.  Its reference is fp64 autograd evaluated at the device
    # forward's own intermediates (afau_grads_anchored: the device's branch decisions, exact
    # arithmetic), gated at 2e-3 of the group's gradient scale.
    assert len(captured) == 1
    ks_dev, sv = captured[0]
    afk = [k for k in net._afau_names]
    tgt = (gt.reshape(len(n1), -1).sum(-1) / torch.minimum(torch.tensor(n1), torch.tensor(n2)).float()).to(DEV)
    dks = 2.0 * 50.0 * (ks_dev.double() - tgt.double()) / len(n1)            # d ks_loss / d ks (mse * K_FACTOR)
    ref_a = afau_grads_anchored(sv, lambda k: pd[k], dks, afk)
    ascale = max(float(v.abs().max()) for v in ref_a.values() if v is not None)
    for k in afk:
        if ref_a[k] is None or float(ref_a[k].abs().max()) == 0.0:
            assert pd[k].grad is None or float(pd[k].grad.abs().max()) < 1e-6 * ascale, k
            errs.pop(k, None)
            continue
        errs[k] = _rel(pd[k].grad, ref_a[k], 1e-3 * ascale)
        assert k.endswith(ZERO_GRAD) or errs[k] < 2e-3, (k, errs[k])
    bd = dict(net.named_buffers())
    for k in sd:
        if "running_" in k:
            assert (bd[k].cpu() - sdl[k]).abs().max() < 1e-5, k
    return errs


# Parameters whose exact gradient is zero: a bias in front of a shift-invariant op (the GNN
# classifiers' bias feeds a Sinkhorn; multi_head_combine.bias feeds an InstanceNorm, which removes
# per-channel shifts).  Both sides return cancellation noise there, so the check is that the
# noise is small against the parameter group's gradient scale.
ZERO_GRAD = ("classifier.bias", "multi_head_combine.bias")


# SplineConv weights: the max aggregation's argmax and the ReLU make their gradient piecewise in
# the inputs; at fp32 resolution the CPU and GPU forwards can route a few (node, channel) maxima
# to different edges.  Measured on the oracle itself: a 1e-6 relative perturbation of one spline
# weight moves the spline weight gradients by 0.7-6% (ragged case).  Their backward is gated at
# 1e-4 by test_spline_layers_bwd_vs_autograd on identical inputs; end to end they get SPLINE_TOL.
SPLINE_TOL = 0.1
# Everything else end to end: the MatchClassifier's backward runs MIOpen convolutions whose
# algorithm (and so rounding) is chosen per run, and the tau = 0.01 Sinkhorn backwards amplify
# such fp32 differences on their way into the GNN; measured 1e-3 .. 5.4e-3 across boxes.
E2E_TOL = 1e-2


def _check_errs(errs, tol):
    zero = {k: v for k, v in errs.items() if k.endswith(ZERO_GRAD) and not k.startswith("classifier")}
    spl = {k: v for k, v in errs.items() if k.startswith(params.SPLINE_PREFIX)}
    assert not spl or max(spl.values()) < SPLINE_TOL, spl
    rest = {k: v for k, v in errs.items() if k not in zero and k not in spl}
    worst = max(rest.values())
    print("train-step relative gradient errors: worst %.2e" % worst, sorted(rest.items(), key=lambda t: -t[1])[:6])
    assert worst < tol, sorted(rest.items(), key=lambda t: -t[1])[:6]
    return zero


def test_train_step_vs_oracle(sd):
    """One training step (PermutationLoss(ds_mat) + ks_loss + cls_loss, training_loop.py:32-60):
    every parameter gradient against autograd through the fp32 oracle."""
    errs = _train_step_compare(synth.make_batch(21, 2, 32), sd, torch.tensor([1.0, 0.0]))
    _check_errs(errs, E2E_TOL)
    assert len(errs) >= 60


def test_train_step_ragged_vs_oracle(sd):
    errs = _train_step_compare(synth.make_batch(22, 3, [30, 24, 28], n2=[26, 30, 28]), sd, torch.tensor([1.0, 0.0, 1.0]))
    _check_errs(errs, E2E_TOL)


def test_train_step_bf16_finite(sd):
    """bf16 operand mode: the step runs and every gradient is finite (reported, not gated)."""
    pairs = synth.make_batch(23, 2, 48)
    gt, n1, n2 = _gt(pairs)
    net = fpm.Net(regression=True, backbone=False, dtype="bf16")
    net.load_state_dict(sd)
    net.to(DEV).train()
    out = net({"fpm_batch": DeviceBatch.from_pairs(pairs, DEV), "gt_perm_mat": gt, "label": torch.ones(2)})
    loss = train.permutation_loss(out["ds_mat"], gt, n1, n2) + out["ks_loss"] + out["cls_loss"]
    loss.backward()
    for k, p in net.named_parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all(), k


@pytest.mark.parametrize("x3", [False, True])
@pytest.mark.parametrize("n1s,n2s", [((40, 40, 40, 40), (40, 40, 40, 40)), ((37, 40, 25, 40), (40, 31, 40, 31))])
def test_afau_hip_backward_vs_replay(sd, n1s, n2s, x3):
    """The hand-written AFA-U backward (fpm.afau_grad / csrc/afau_bwd.hip) against autograd through
    the device statement of the regressor (fpm.afau_torch, pinned to the oracle in float64 by
    tests/test_train_cpu.py) at the same ss and d(ks): every regressor parameter, relative to its
    group's gradient scale.  Zero-gradient parameters (Wq, Wk, the dot-product row of mix1, the col
    block's attention, combine biases in front of an instance norm) are exactly 0 here.  ``x3``: the
    regressor's GEMMs on split bf16x3 operands (the bf16 training mode), same gates."""
    import os
    from fpm import afau_torch, afau_grad
    g = torch.Generator().manual_seed(sum(n1s) + sum(n2s))
    B, n1max, n2max = len(n1s), max(n1s), max(n2s)
    ss = torch.zeros(B, n1max, n2max)
    for b in range(B):
        ss[b, :n1s[b], :n2s[b]] = torch.softmax(torch.randn(n1s[b], n2s[b], generator=g) * 3, dim=1)
    pairs = synth.make_batch(5, B, list(n1s), n2=list(n2s))
    bt = DeviceBatch.from_pairs(pairs, DEV)
    names = [k for k in sd if k.startswith(afau_torch.AFAU_PARAM_PREFIXES) and sd[k].is_floating_point()]
    prm = {k: sd[k].to(DEV).float() for k in names}
    ssd = ss.to(DEV)
    ks, sv = afau_grad.forward(lambda k: prm[k], ssd, bt, x3=x3)
    dks = torch.randn(B, generator=g).to(DEV)
    grads = dict(zip(names, afau_grad.backward(lambda k: prm[k], sv, dks, names)))
    leaves = {k: v.clone().requires_grad_(True) for k, v in prm.items()}
    ks_ref = afau_torch.afau_ks(ssd, torch.tensor(n1s, device=DEV), torch.tensor(n2s, device=DEV),
                                lambda k: leaves[k])
    assert (ks - ks_ref).abs().max() < 1e-5
    (ks_ref * dks).sum().backward()
    scale = {}
    for k in names:
        grp = k.split(".")[0] + ("." + k.split(".")[3] if k.startswith("encoder_k") else "")
        if leaves[k].grad is not None:
            scale[grp] = max(scale.get(grp, 0.0), float(leaves[k].grad.abs().max()))
    for k in names:
        grp = k.split(".")[0] + ("." + k.split(".")[3] if k.startswith("encoder_k") else "")
        ref = leaves[k].grad
        got = grads[k].cpu()
        if ref is None or k.endswith(("Wq.weight", "Wk.weight")):
            assert float(got.abs().max()) == 0.0, k
            continue
        tol = 2e-3 * max(scale[grp], 1e-12)
        err = float((got - ref.cpu()).abs().max())
        assert err <= tol or k.endswith("multi_head_combine.bias"), (k, err, tol)


def test_outer_sum_kernel():
    """fpm_outer_sum (GNN weight / bias gradient reductions) against the float64 sums, incl. strided
    channel views and a ragged slice count."""
    from fpm.train import _outer_sum
    g = torch.Generator().manual_seed(44)
    for B, O, Cc, N in ((3, 16, 17, 10000), (2, 1, 16, 65536), (4, 16, 1, 333), (2, 32, 17, 9000), (3, 20, 5, 4097)):
        U = torch.randn(B, O + 1, N, generator=g)[:, 1:]          # strided channel view
        V = torch.randn(B, Cc, N, generator=g)
        w, bsum = _outer_sum(U.to(DEV), V.to(DEV), ones=True)
        ref = torch.einsum("bon,bcn->oc", U.double(), V.double())
        assert (w.cpu().double() - ref).abs().max() < 1e-4 * ref.abs().max()
        assert (bsum.cpu().double() - U.double().sum((0, 2))).abs().max() < 1e-6 * float(U.abs().sum())
        assert torch.equal(_outer_sum(U.to(DEV), V.to(DEV)), w)
        # the 16-B staging variant (aligned rows, N % 4 == 0) against the 4-B one: same bits
        prev = ops.set_tuning("outer_sum_vec", 0)
        try:
            w0, b0 = _outer_sum(U.to(DEV), V.to(DEV), ones=True)
        finally:
            ops.set_tuning("outer_sum_vec", prev)
        assert torch.equal(w0, w) and torch.equal(b0, bsum)
        if O == 32:
            # the fused [dx1; dh1] form: each 16-row half equals its own call bit for bit
            for h in (slice(0, 16), slice(16, 32)):
                wh, bh = _outer_sum(U[:, h].to(DEV), V.to(DEV), ones=True)
                assert torch.equal(wh, w[h]) and torch.equal(bh, bsum[h])


@pytest.mark.parametrize("shape,off", [((4, 16, 64, 64), 0.0), ((3, 32, 17, 19), 0.0), ((4, 16, 64, 64), 100.0)])
def test_bn_relu_train_vs_torch(shape, off):
    """HIP BatchNorm2d(relu(x)) in train mode vs torch F.relu + F.batch_norm(training=True):
    output, running buffers and the gradients of x, gamma, beta (ngm.py:90-99).  ``off``: a large
    per-channel offset (|mean| >> std), where E[r^2] - mean^2 would cancel."""
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(*shape, generator=g) + off * (1.0 + torch.rand(shape[1], generator=g))[None, :, None, None]
    gamma = torch.rand(shape[1], generator=g) + 0.5
    beta = torch.randn(shape[1], generator=g) * 0.1
    gy = torch.randn(*shape, generator=g)
    rm0, rv0 = torch.randn(shape[1], generator=g) * 0.1, torch.rand(shape[1], generator=g) + 0.5
    # torch reference (float64 on CPU)
    xr, gr, br = (t.double().clone().requires_grad_(True) for t in (x, gamma, beta))
    rmr, rvr = rm0.double().clone(), rv0.double().clone()
    yr = F_.batch_norm(F_.relu(xr), rmr, rvr, gr, br, True, 0.1, 1e-5)
    (yr * gy.double()).sum().backward()
    # HIP
    xd, gd, bd = (t.to(DEV).clone().requires_grad_(True) for t in (x, gamma, beta))
    rmd, rvd = rm0.to(DEV).clone(), rv0.to(DEV).clone()
    y = train.BnReluFn.apply(xd, gd, bd, rmd, rvd, 0.1, 1e-5)
    (y * gy.to(DEV)).sum().backward()
    assert _rel(y, yr.detach()) < 1e-5
    assert _rel(rmd, rmr) < 1e-5 and _rel(rvd, rvr) < 1e-5
    assert _rel(xd.grad, xr.grad) < 1e-4
    assert _rel(gd.grad, gr.grad) < 1e-4 and _rel(bd.grad, br.grad) < 1e-4


@pytest.mark.parametrize("op", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("fwd", [True, False])
def test_spline_weight_pack_exact(op, fwd):
    """fpm_spline_weight_pack equals the torch transpose / cat / cast it replaces, bit for bit
    (odd sizes: partial 64 x 64 tiles)."""
    g = torch.Generator().manual_seed(3)
    weight = torch.randn(25, 70, 97, generator=g).to(DEV)
    root = torch.randn(70, 97, generator=g).to(DEV)
    os.environ["FPM_SPLINE_WPACK"] = "hip"
    try:
        got = train._spline_w({}, weight, root, op, fwd)
    finally:
        os.environ.pop("FPM_SPLINE_WPACK", None)
    if fwd:
        ref = torch.cat([weight.transpose(1, 2), root.t()[None]]).contiguous().to(op)
    else:
        ref = torch.cat([weight, root[None]]).contiguous().to(op)
    assert got.shape == ref.shape and got.dtype == ref.dtype
    assert torch.equal(got, ref)


def _cls_ref_train(s, perm, prm, bufs):
    """MatchClassifier (ngm.py:75-106) in train mode, torch float64 on the CPU (the gradient reference)."""
    w1, b1, g1, be1, w2, b2, g2, be2, fcw, fcb = prm
    rm1, rv1, rm2, rv2 = bufs
    x = (s * perm).unsqueeze(1)
    x = F_.batch_norm(F_.relu(F_.conv2d(x, w1, b1, padding=1)), rm1, rv1, g1, be1, True, 0.1, 1e-5)
    x = F_.max_pool2d(x, 2)
    x = F_.batch_norm(F_.relu(F_.conv2d(x, w2, b2, padding=1)), rm2, rv2, g2, be2, True, 0.1, 1e-5)
    x = F_.max_pool2d(x, 2)
    x = F_.adaptive_avg_pool2d(x, 1).view(x.shape[0], -1)
    return F_.linear(x, fcw, fcb).squeeze(-1)


@pytest.mark.parametrize("B,H,W,dense", [(2, 37, 29, True), (3, 64, 48, True), (2, 5, 4, True), (4, 256, 256, False),
                                         (2, 131, 97, False), (1, 40, 33, True), (1, 63, 70, False)])
def test_match_cls_train_fused_vs_torch(B, H, W, dense):
    """The fused train-mode MatchClassifier (fpm_match_cls_train_fwd / _bwd) against torch autograd in
    float64: logits, both BatchNorms' running buffers, d/ds and every parameter gradient.  Odd map sizes
    exercise the conv positions outside every pooling window (in the BN statistics and the backward);
    ``dense``: perm all ones (continuous activations), else a sparse match mask (the training case:
    most windows tie exactly at relu(bias), MaxPool routes to the first).  Tolerance 1e-4 of each
    gradient's scale (fp32 sums over up to 2^20 positions against float64)."""
    g = torch.Generator().manual_seed(B * 1000 + H + W)
    s = torch.rand(B, H, W, generator=g)
    if dense:
        perm = torch.ones(B, H, W)
    else:
        perm = torch.zeros(B, H, W)
        for b in range(B):
            k = min(H, W)
            perm[b, torch.randperm(H, generator=g)[:k], torch.randperm(W, generator=g)[:k]] = 1.0
    prm = [torch.randn(16, 1, 3, 3, generator=g) * 0.5, torch.randn(16, generator=g) * 0.1,
           torch.rand(16, generator=g) + 0.5, torch.randn(16, generator=g) * 0.1,
           torch.randn(32, 16, 3, 3, generator=g) * 0.2, torch.randn(32, generator=g) * 0.1,
           torch.rand(32, generator=g) + 0.5, torch.randn(32, generator=g) * 0.1,
           torch.randn(1, 32, generator=g), torch.randn(1, generator=g)]
    bufs = [torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5,
            torch.randn(32, generator=g) * 0.1, torch.rand(32, generator=g) + 0.5]
    gl = torch.randn(B, generator=g)
    sr = s.double().clone().requires_grad_(True)
    pr = [p.double().clone().requires_grad_(True) for p in prm]
    br = [t.double().clone() for t in bufs]
    lr = _cls_ref_train(sr, perm.double(), pr, br)
    (lr * gl.double()).sum().backward()
    sd_ = s.to(DEV).clone().requires_grad_(True)
    pd = [p.to(DEV).clone().requires_grad_(True) for p in prm]
    bd = [t.to(DEV).clone() for t in bufs]
    ld = train.MatchClsTrainFn.apply(sd_, perm.to(DEV), *pd, *bd, 0.1, 1e-5)
    (ld * gl.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert _rel(ld, lr.detach()) < 1e-5
    for a, b_ in zip(bd, br):
        assert _rel(a, b_) < 1e-5
    assert _rel(sd_.grad, sr.grad) < 1e-4
    names = ["w1", "b1", "g1", "be1", "w2", "b2", "g2", "be2", "fcw", "fcb"]
    for nm, a, b_ in zip(names, pd, pr):
        assert a.grad is not None and a.grad.shape == b_.shape, nm
        assert _rel(a.grad, b_.grad) < 1e-4, (nm, _rel(a.grad, b_.grad))


def test_match_cls_train_fused_deterministic():
    """Two runs of the fused train-mode classifier give bit-identical outputs and gradients (every
    reduction is in a fixed order)."""
    g = torch.Generator().manual_seed(7)
    B, H, W = 3, 96, 80
    s = torch.rand(B, H, W, generator=g).to(DEV)
    perm = (torch.rand(B, H, W, generator=g) > 0.7).float().to(DEV)
    prm = [torch.randn(16, 1, 3, 3, generator=g), torch.randn(16, generator=g), torch.rand(16, generator=g) + 0.5,
           torch.randn(16, generator=g), torch.randn(32, 16, 3, 3, generator=g) * 0.2, torch.randn(32, generator=g),
           torch.rand(32, generator=g) + 0.5, torch.randn(32, generator=g), torch.randn(1, 32, generator=g),
           torch.randn(1, generator=g)]
    outs = []
    for _ in range(2):
        sd_ = s.clone().requires_grad_(True)
        pd = [p.to(DEV).clone().requires_grad_(True) for p in prm]
        bd = [torch.zeros(16, device=DEV), torch.ones(16, device=DEV), torch.zeros(32, device=DEV),
              torch.ones(32, device=DEV)]
        ld = train.MatchClsTrainFn.apply(sd_, perm, *pd, *bd, 0.1, 1e-5)
        ld.sum().backward()
        outs.append([ld.detach(), sd_.grad] + [p.grad for p in pd] + bd)
    for a, b_ in zip(*outs):
        assert torch.equal(a, b_)


def test_spline_scatter_bwd_matches_atomic(sd):
    """At the C3 graph size (n = 256 Delaunay, bf16 operands) the scatter backward's input and
    weight gradients equal the atomic form's up to summation order (the fp32 parity of both forms
    against the oracle is test_spline_layers_bwd_vs_autograd)."""
    pairs = synth.make_batch(19, 4, 256)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    pre = params.SPLINE_PREFIX
    res = {}
    for scatter in ("1", "0"):
        os.environ["FPM_SPLINE_SCATTER"] = scatter
        try:
            side = train._Side(bt, 1)
            W = {k: sd[k].clone().to(DEV).requires_grad_(True) for k in sd if k.startswith(pre) and sd[k].is_floating_point()}
            x0 = bt.x[1].clone().requires_grad_(True)
            h = train.SplineLayerFn.apply(x0, W[pre + ".0.weight"], W[pre + ".0.root"], W[pre + ".0.bias"], None, side, 0,
                                          "bf16")
            o = train.SplineLayerFn.apply(h, W[pre + ".1.weight"], W[pre + ".1.root"], W[pre + ".1.bias"], x0, side, 1,
                                          "bf16")
            R = torch.randn(o.shape, generator=torch.Generator().manual_seed(4)).to(DEV)
            (o * R).sum().backward()
            res[scatter] = [x0.grad.clone()] + [W[k].grad.clone() for k in sorted(W)]
        finally:
            os.environ.pop("FPM_SPLINE_SCATTER", None)
    # fp32 product-row gradients summed in another order, then rounded to bf16 for the grouped
    # GEMM and the bf16 weight-gradient products: agreement at the bf16 ulp scale (2^-8)
    for a, b in zip(res["1"], res["0"]):
        assert _rel(a, b) < 1e-2


def test_spline_scatter_bwd_batches_bit_identical(sd):
    """The scatter backward's out-edge load batches (fpm_set_tuning "scatter_batch" 4, the default)
    give the same gradients bit for bit as one edge at a time (1): same sums in the same order.
    Also with the fp32 cell rows written ("scatter_f32_rows" 1): nothing downstream reads them."""
    pairs = synth.make_batch(23, 4, 256)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    pre = params.SPLINE_PREFIX
    res = []
    for qb, f32rows in ((1, 0), (4, 0), (4, 1)):
        prev = [(k, ops.set_tuning(k, v)) for k, v in (("scatter_batch", qb), ("scatter_f32_rows", f32rows))]
        try:
            side = train._Side(bt, 0)
            W = {k: sd[k].clone().to(DEV).requires_grad_(True) for k in sd if k.startswith(pre) and sd[k].is_floating_point()}
            x0 = bt.x[0].clone().requires_grad_(True)
            h = train.SplineLayerFn.apply(x0, W[pre + ".0.weight"], W[pre + ".0.root"], W[pre + ".0.bias"], None, side, 0,
                                          "bf16")
            o = train.SplineLayerFn.apply(h, W[pre + ".1.weight"], W[pre + ".1.root"], W[pre + ".1.bias"], x0, side, 1,
                                          "bf16")
            R = torch.randn(o.shape, generator=torch.Generator().manual_seed(5)).to(DEV)
            (o * R).sum().backward()
            res.append([x0.grad.clone()] + [W[k].grad.clone() for k in sorted(W)])
        finally:
            for k, v in prev:
                ops.set_tuning(k, v)
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert torch.equal(a, b)


def test_train_second_net_uses_its_own_weights():
    """Two Nets trained one after the other in one process (the second from another seed, loaded
    with load_state_dict, and one weight changed in place through ``.data``): each training
    forward uses its own current SplineConv weights (the operand copies live for one step only)."""
    pairs = synth.make_batch(24, 2, 32)
    gt, n1, n2 = _gt(pairs)
    for seed in (7, 8):
        sdx = params.init_params(seed)
        net = fpm.Net(regression=True, backbone=False, dtype="f32")
        net.load_state_dict(sdx)
        net.to(DEV).train()
        for step in range(2):
            if step == 1:      # in-place update that does not bump _version
                p = dict(net.named_parameters())[params.SPLINE_PREFIX + ".0.weight"]
                p.data.mul_(1.25)
                sdx[params.SPLINE_PREFIX + ".0.weight"] = p.detach().cpu().clone()
            out = net({"fpm_batch": DeviceBatch.from_pairs(pairs, DEV), "gt_perm_mat": gt, "label": torch.ones(2)})
            (train.permutation_loss(out["ds_mat"], gt, n1, n2) + out["ks_loss"]).backward()
            ref = O.forward(pairs, sdx, regression=True, training=True, gt_perm=gt, labels=torch.ones(2))
            assert (net.last_outputs["ss"].detach().cpu() - ref["ss"].detach()).abs().max() < 1e-4, (seed, step)
        del net


@pytest.mark.gpu
def test_rows_sum_vector_path_bitwise():
    """fpm_rows_sum's 16-B path (K % 4 == 0, aligned rows) gives the same bits as its scalar path (a
    view shifted by one float), with and without keys, and equals the in-order float32 sum."""
    from fpm.afau_grad import rows_sum
    g = torch.Generator().manual_seed(7)
    for B, K in ((64, 4096), (300, 768), (5, 12)):
        x = torch.randn(B, K, generator=g)
        xa = x.to(DEV)
        buf = torch.empty(B * K + 1, device=DEV)
        buf[1:].copy_(xa.reshape(-1))
        xm = buf[1:].view(B, K)                                  # 4-B offset: scalar path
        assert xm.data_ptr() % 16 != 0
        ra, rm = rows_sum(xa), rows_sum(xm)
        assert torch.equal(ra, rm)
        if B <= 256:
            ref = torch.zeros(K)
            for b in range(B):
                ref = ref + x[b]
            assert torch.equal(ra.cpu(), ref)
        key = torch.randint(0, 3, (B,), generator=g, dtype=torch.int32).to(DEV)
        assert torch.equal(rows_sum(xa, key=key, nkeys=3), rows_sum(xm, key=key, nkeys=3))


def test_gather_transpose_bf16_paths():
    """fpm_gather_transpose (bf16): the 16-B path (Q, ldo multiples of 8) and the 32-bit path (ldo =
    Q + 2) both give out[c][q] = in[rows[q]][c] (0 for rows[q] < 0), bit for bit."""
    from fpm import _lib
    g = torch.Generator().manual_seed(11)
    R, C, Q = 300, 128, 200
    x = torch.randn(R, C, generator=g).to(torch.bfloat16).to(DEV)
    rows = torch.randint(-1, R, (Q,), generator=g, dtype=torch.int32).to(DEV)
    ref = torch.where(rows.long()[None, :] >= 0, x[rows.long().clamp(min=0)].t(), torch.zeros((), dtype=x.dtype, device=DEV))
    for ldo in (Q, Q + 2):
        out = torch.full((C, ldo), 7.0, dtype=torch.bfloat16, device=DEV)
        _lib.call("fpm_gather_transpose", 1, ops._p(x), x.stride(0), ops._p(rows), Q, C, ops._p(out), ldo,
                  ops._stream(x))
        torch.cuda.synchronize()
        assert torch.equal(out[:, :Q], ref), ldo


def test_perm_loss_kernel_vs_reference_loop():
    """The fused device PermutationLoss (fpm_perm_loss_fwd / _bwd, src/loss_func.py:26-59) against
    the reference's per-pair BCE loop under autograd: ragged pairs, saturated entries (ds = 0 / 1
    exactly: the clamped logs and the 1e-12 floor of the backward), padding ignored."""
    g = torch.Generator().manual_seed(13)
    B, n1max, n2max = 5, 40, 37
    n1 = [40, 33, 17, 40, 25]
    n2 = [37, 37, 30, 12, 37]
    ds = torch.rand(B, n1max, n2max, generator=g) * 0.98 + 0.01
    ds[0, 0, 0], ds[1, 3, 4], ds[2, 1, 1] = 0.0, 1.0, 1e-30
    gt = torch.zeros(B, n1max, n2max)
    for b in range(B):
        k = min(n1[b], n2[b])
        gt[b, torch.arange(k), torch.randperm(n2[b], generator=g)[:k]] = 1.0
    gt[1, 3, 4] = 1.0
    ref_ds = ds.clone().double().requires_grad_(True)
    ref = O.permutation_loss(ref_ds, gt.double(), n1, n2)
    ref.backward()
    dev_ds = ds.to(DEV).requires_grad_(True)
    loss = train.permutation_loss(dev_ds, gt.to(DEV), n1, n2)
    (loss * 1.7).backward()
    assert abs(float(loss) - float(ref)) < 1e-5 * max(1.0, abs(float(ref))), (float(loss), float(ref))
    gd, gr = dev_ds.grad.cpu().double(), ref_ds.grad * 1.7
    fin = torch.isfinite(gr) & (gr.abs() < 1e6)
    assert (gd[fin] - gr[fin]).abs().max() <= 1e-5 * gr[fin].abs().max(), float((gd[fin] - gr[fin]).abs().max())
    for b in range(B):
        assert gd[b, n1[b]:].abs().max() == 0 if n1[b] < n1max else True
        assert gd[b, :, n2[b]:].abs().max() == 0 if n2[b] < n2max else True


def test_perm_loss_kernel_clamps_sizes_and_checks_range():
    """sizes beyond the padded box are clamped like the reference's slice
    ds[b, :n1, :n2] (never reading the next pair), and a ds / gt entry outside [0, 1] or NaN raises
    like the reference's assert (loss_func.py:42-47)."""
    from fpm._lib import FpmError
    g = torch.Generator().manual_seed(3)
    B, n1max, n2max = 3, 9, 7
    ds = (torch.rand(B, n1max, n2max, generator=g) * 0.9 + 0.05).to(DEV)
    gt = (torch.rand(B, n1max, n2max, generator=g) > 0.8).float().to(DEV)
    big = torch.tensor([50, 9, 4], dtype=torch.int32, device=DEV)
    clamped = torch.tensor([9, 9, 4], dtype=torch.int32, device=DEV)
    n2 = torch.tensor([7, 100, 7], dtype=torch.int32, device=DEV)
    n2c = torch.tensor([7, 7, 7], dtype=torch.int32, device=DEV)
    a = ops.perm_loss_fwd(ds, gt, big, n2)
    # the reference's loop slices (clamps) each block and divides by sum(n1) as given
    ref = O.permutation_loss(ds.cpu().double(), gt.cpu().double(), [50, 9, 4], [7, 100, 7])
    assert abs(float(a) - float(ref)) < 1e-5 * float(ref), (float(a), float(ref))
    b_ = ops.perm_loss_fwd(ds, gt, clamped, n2c)
    assert abs(float(a) * 63 - float(b_) * 22) < 1e-5 * float(b_) * 22
    for bad_val in (1.5, -0.25, float("nan")):
        d2 = ds.clone()
        d2[1, 2, 3] = bad_val
        with pytest.raises(FpmError, match="outside"):
            ops.perm_loss_fwd(d2, gt, clamped, n2c)
    d2 = ds.clone()
    d2[2, 6, 6] = 7.0                       # outside pair 2's 4 x 7 block: ignored
    ops.perm_loss_fwd(d2, gt, clamped, n2c)
    # check_range = N accumulates the flags on the device and reads them every N-th call
    d2 = ds.clone()
    d2[0, 0, 0] = 2.0
    ops.perm_loss_fwd(d2, gt, clamped, n2c, check_range=3)
    ops.perm_loss_fwd(ds, gt, clamped, n2c, check_range=3)
    with pytest.raises(FpmError, match="1 pair"):
        ops.perm_loss_fwd(ds, gt, clamped, n2c, check_range=3)
    ops.perm_loss_fwd(d2, gt, clamped, n2c, check_range=0)      # off
