"""Diagnostic of the AFA-U k deviation on the image-path test inputs: GPU vs fp32 / float64 CPU
oracle, with and without the score LUT, and the regressor alone on the oracle's ss."""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.getcwd() + "/tests")
import torch, numpy as np
import fpm
from fpm import ops, params
from fpm.batch import DeviceBatch
import oracle as O
from oracle import graphs_oracle as GO
from test_frontend import _image_batch
DEV = torch.device("cuda", 0)
net = fpm.Net(regression=True, backbone=True)
sd = params.init_params(5)
net.load_state_dict({**net.state_dict(), **sd})
B, n = 3, 32
imgs, Ps, ns = _image_batch(B, n, 8)
xs, gs = net.image_features(imgs, Ps, ns, DEV)
pairs = []
for b in range(B):
    pr = []
    for side in range(2):
        m = int(ns[side][b]); p = Ps[side][b, :m].numpy()
        A = GO.delaunay_triangulate(p.astype(np.float64)); ei, attr = GO.pyg_edges(A, p)
        x = xs[side].view(B, n, -1)[b, :m].cpu().numpy()
        pr.append(dict(n=m, x=x, w=gs[side][b].cpu().numpy(), edge_index=ei, pseudo=attr, P=p, A=A))
    pairs.append(tuple(pr))
orc = O.forward(pairs, {k: v for k, v in net.state_dict().items()})
for lut in (1, 0):
    ops.set_tuning("afau_lut", lut)
    ref = net.run(DeviceBatch.from_pairs(pairs, DEV))
    print("lut", lut, "ss", float((ref["ss"].cpu() - orc["ss"]).abs().max()), "k", (ref["k_prob"].cpu() - orc["k_prob"]).abs().tolist())
    # AFA-U on the oracle's ss
    bt = DeviceBatch.from_pairs(pairs, DEV)
    ks = net._afau(net.packed(DEV), orc["ss"].to(DEV).contiguous(), bt)
    print("   afau on oracle ss: k diff", (ks.cpu() - orc["k_prob"]).abs().tolist())
sdd = {k: (v.double() if v.is_floating_point() else v) for k, v in net.state_dict().items()}
o64 = O.forward(pairs, sdd, dtype=torch.float64)
ops.set_tuning("afau_lut", 2)
ref = net.run(DeviceBatch.from_pairs(pairs, DEV))
print("vs f64 oracle: gpu k", (ref["k_prob"].cpu().double() - o64["k_prob"]).abs().tolist(),
      "fp32 oracle k", (orc["k_prob"].double() - o64["k_prob"]).abs().tolist())
