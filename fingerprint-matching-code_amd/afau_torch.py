"""Differentiable PyTorch (device) statement of the AFA-U k regressor, used only by the training
backward: the forward value always comes from the HIP kernels (``Net._afau``); ``train.AfauFn``
replays this graph under autograd to obtain the encoder / head gradients of ``ks_loss``
(``src/model/afau.py:54-300``, ``ngm.py:386-412``; ``ss`` is detached there, ngm.py:398, so no
gradient leaves the regressor).  Runs on the tensors' device (GPU in the product path).
"""
import math

import torch
import torch.nn.functional as F

from . import config as C


def _block(a, bemb, cost, g):
    """EncodingBlock.forward (afau.py:109-142) with CrossSet_MultiHeadAttention (:231-300)."""
    B, R, _ = a.shape
    Cn = bemb.shape[1]
    H, D = C.AFAU_HEADS, C.AFAU_QKV
    q = F.linear(a, g("Wq.weight")).view(B, R, H, D).transpose(1, 2)          # (B, H, R, D)
    k = F.linear(bemb, g("Wk.weight")).view(B, Cn, H, D).transpose(1, 2)
    v = F.linear(bemb, g("Wv.weight")).view(B, Cn, H, D).transpose(1, 2)
    dot = torch.matmul(q, k.transpose(2, 3)) / C.AFAU_SQRT_QKV                 # (B, H, R, Cn)
    w1 = g("mixed_score_MHA.mix1_weight")                                      # (H, 2, MS)
    b1 = g("mixed_score_MHA.mix1_bias")                                        # (H, MS)
    w2 = g("mixed_score_MHA.mix2_weight")                                      # (H, MS, 1)
    b2 = g("mixed_score_MHA.mix2_bias")                                        # (H, 1)
    # mixed score per head: relu([dot, cost] W1_h + b1_h) W2_h + b2_h, in the reference's matmul
    # form (afau.py:245-262).  Its rounding matters: the regressor's gradient jumps at the ReLU
    # kinks and the max pool, so a reordered sum (e.g. one hidden unit at a time) lands on other
    # branches for some entries and moves the FFN gradients by O(10 %).
    two = torch.stack((dot, cost[:, None].expand_as(dot)), dim=4).transpose(1, 2)   # (B, R, H, Cn, 2)
    ms1 = torch.matmul(two, w1) + b1[None, None, :, None, :]
    mixed = (torch.matmul(F.relu(ms1), w2) + b2[None, None, :, None, :]).transpose(1, 2).squeeze(4)
    att = torch.softmax(mixed, dim=3)
    out = torch.matmul(att, v).transpose(1, 2).reshape(B, R, H * D)
    mh = F.linear(out, g("multi_head_combine.weight"), g("multi_head_combine.bias"))
    o1 = _inorm(a + mh, g("add_n_normalization_1.norm.weight"), g("add_n_normalization_1.norm.bias"))
    ff = F.linear(F.relu(F.linear(o1, g("feed_forward.W1.weight"), g("feed_forward.W1.bias"))),
                  g("feed_forward.W2.weight"), g("feed_forward.W2.bias"))
    return _inorm(o1 + ff, g("add_n_normalization_2.norm.weight"), g("add_n_normalization_2.norm.bias"))


def _inorm(x, w, b):
    """AddAndInstanceNormalization (afau.py:154-176): InstanceNorm1d over positions, affine."""
    return F.instance_norm(x.transpose(1, 2), weight=w, bias=b, eps=C.IN_EPS).transpose(1, 2)


def afau_ks(ss, n1, n2, P):
    """ks (B,) from the doubly-stochastic ``ss`` (B, n1max, n2max); ``P(name)`` returns the
    parameter ``name`` (reference state_dict names)."""
    B, n1max, n2max = ss.shape
    dev, dt = ss.device, ss.dtype
    row0 = torch.zeros(B, n1max, C.UNIV_SIZE, device=dev, dtype=dt)
    idx = torch.arange(n2max, device=dev)
    col0 = ((idx[None, :, None] == torch.arange(C.UNIV_SIZE, device=dev)[None, None, :])
            & (idx[None, :, None] < n2.to(dev).view(-1, 1, 1))).to(dt)          # one-hot rows (ngm.py:391-395)
    pre = "encoder_k.layers.0."
    r = _block(row0, col0, ss, lambda k: P(pre + "row_encoding_block." + k))
    # the column block reads one-hot rows against zero rows (k = v = 0): it depends on n2 only, so
    # it runs once per distinct n2 and is gathered (gradients sum over the pairs sharing it)
    n2c = n2.to(dev).view(-1)
    n2u, inv = torch.unique(n2c, return_inverse=True)
    col0u = ((idx[None, :, None] == torch.arange(C.UNIV_SIZE, device=dev)[None, None, :])
             & (idx[None, :, None] < n2u.view(-1, 1, 1))).to(dt)
    row0u = torch.zeros(n2u.numel(), n1max, C.UNIV_SIZE, device=dev, dtype=dt)
    costu = torch.zeros(n2u.numel(), n2max, n1max, device=dev, dtype=dt)     # unused: v = 0
    c = _block(col0u, row0u, costu, lambda k: P(pre + "col_encoding_block." + k))
    gr = r.max(dim=1).values        # pad to UNIV_SIZE with -inf + MaxPool1d (ngm.py:401-404)
    gc = c.max(dim=1).values[inv]
    kr = F.linear(F.relu(F.linear(gr, P("final_row.0.weight"), P("final_row.0.bias"))),
                  P("final_row.2.weight"), P("final_row.2.bias")).squeeze(-1)
    kc = F.linear(F.relu(F.linear(gc, P("final_col.0.weight"), P("final_col.0.bias"))),
                  P("final_col.2.weight"), P("final_col.2.bias")).squeeze(-1)
    return torch.sigmoid((kr + kc) / 2)


AFAU_PARAM_PREFIXES = ("encoder_k.", "final_row.", "final_col.")
