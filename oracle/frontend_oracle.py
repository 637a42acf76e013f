"""CPU restatement of the image front end of ``Net.forward`` — TEST ORACLE ONLY (see ``oracle/__init__``).

``src/model/ngm.py:235-248``: global = AdaptiveMaxPool2d(1)(edges) (``ResNet18_final.final_layers``,
``feature_extractor.py:62``), ``normalize_over_channels`` (ngm.py:65-67), ``feature_align``
(``utils/feature_align.py:5-126``, vectorised over points with the reference's fp32 operation
order, incl. the (H, W) vs (320, 240) scale mix and the border nearest-neighbour branch) and
``concat_features`` (ngm.py:70-72).  Pinned by ``tests/golden/feature_align.npz`` (generated from
the reference's own ``utils.feature_align``).
"""
import torch


def normalize_over_channels(x):
    """ngm.py:65-67."""
    return x / torch.norm(x, dim=1, keepdim=True)


def bilinear_points(im, x, y):
    """bilinear_interpolate (feature_align.py:71-126) for vectors of points: im (c, h, w)."""
    x = x.to(torch.float32)
    y = y.to(torch.float32)
    x0 = torch.floor(x)
    x1 = x0 + 1
    y0 = torch.floor(y)
    y1 = y0 + 1
    x0 = torch.clamp(x0, 0, im.shape[2] - 1).to(torch.int64)
    x1 = torch.clamp(x1, 0, im.shape[2] - 1).to(torch.int64)
    y0 = torch.clamp(y0, 0, im.shape[1] - 1).to(torch.int64)
    y1 = torch.clamp(y1, 0, im.shape[1] - 1).to(torch.int64)
    Ia, Ib, Ic, Id = im[:, y0, x0], im[:, y1, x0], im[:, y0, x1], im[:, y1, x1]
    ex = x0 == x1
    ey = y0 == y1
    x0 = torch.where(ex & (x0 == 0), x0 - 1, x0).to(torch.float32)
    x1 = torch.where(ex & (x0 != -1), x1 + 1, x1).to(torch.float32)
    y0 = torch.where(ey & (y0 == 0), y0 - 1, y0).to(torch.float32)
    y1 = torch.where(ey & (y0 != -1), y1 + 1, y1).to(torch.float32)
    wa = (x1 - x) * (y1 - y)
    wb = (x1 - x) * (y - y0)
    wc = (x - x0) * (y1 - y)
    wd = (x - x0) * (y - y0)
    return Ia * wa + Ib * wb + Ic * wc + Id * wd


def feature_align(raw_feature, P, ns, ori_size=(320, 240)):
    """feature_align.py:5-68 -> (b, c, n_max), zeros past ns[b]."""
    b, c = raw_feature.shape[:2]
    n_max = P.shape[1]
    dev = raw_feature.device               # feature_align.py:23-24: output on the input's device
    ori = torch.tensor(ori_size, dtype=torch.float32, device=dev)
    F = torch.zeros(b, c, n_max, dtype=raw_feature.dtype, device=dev)
    P = P.to(dev)
    for idx in range(b):
        n = int(ns[idx])
        feat = raw_feature[idx]
        fs = torch.as_tensor(feat.shape[1:3], dtype=torch.float32, device=dev)
        step = ori / fs
        p = (P[idx, :n].float() - step / 2) / ori * fs
        F[idx, :, :n] = bilinear_points(feat, p[:, 0], p[:, 1])
    return F


def image_features(nodes, edges, P, ns, ori_size=(320, 240)):
    """ngm.py:235-248 after the CNN: per-keypoint [U || F] rows (b, n_max, c_n + c_e) with zero
    padding rows, and the global feature (b, c_e)."""
    glob = torch.amax(edges, dim=(2, 3))
    U = feature_align(normalize_over_channels(nodes), P, ns, ori_size)
    F = feature_align(normalize_over_channels(edges), P, ns, ori_size)
    return torch.cat([U, F], dim=1).transpose(1, 2).contiguous(), glob
