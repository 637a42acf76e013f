"""Diagnose ShardedNet vs Net on the data_dict path: per-output, per-pair max differences for
(a) Net twice (determinism), (b) ShardedNet threaded, (c) ShardedNet with shards run serially."""
import os
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import fpm  # noqa: E402
from fpm import params, synth  # noqa: E402
from fpm.parallel import ShardedNet  # noqa: E402

sd = params.init_params(5)
pairs = synth.make_batch(42, 5, 40, n2=[40, 33, 40, 38, 40])
B = len(pairs)


def dd(gt=True):
    d = {"ns": [torch.tensor([p[s]["n"] for p in pairs]) for s in range(2)], "pyg_graphs": [],
         "node_features": [], "global_features": []}

    class G:
        pass
    for side in range(2):
        g = G()
        offs = np.cumsum([0] + [p[side]["n"] for p in pairs])
        g.edge_index = torch.from_numpy(np.concatenate([p[side]["edge_index"] + offs[b] for b, p in enumerate(pairs)], 1))
        g.edge_attr = torch.from_numpy(np.concatenate([p[side]["pseudo"] for p in pairs]))
        g.ptr = torch.from_numpy(offs)
        d["pyg_graphs"].append(g)
        d["node_features"].append(torch.from_numpy(np.concatenate([p[side]["x"] for p in pairs])))
        d["global_features"].append(torch.from_numpy(np.stack([p[side]["w"] for p in pairs])))
    if gt:
        gtm = torch.zeros(B, 40, 40)
        for b in range(B):
            m = min(pairs[b][0]["n"], pairs[b][1]["n"])
            gtm[b, range(m), range(m)] = 1
        d["gt_perm_mat"] = gtm
        d["label"] = torch.tensor([1.0, 0.0, 1.0, 1.0, 0.0])
    return d


def cmp(tag, a, b):
    for k in ("ds_mat", "perm_mat", "k_prob", "cls_prob"):
        x, y = a[k].float().cpu(), b[k].float().cpu()
        per = [float((x[i] - y[i]).abs().max()) for i in range(B)]
        print(tag, k, "equal" if torch.equal(x, y) else "DIFF", ["%.2e" % v for v in per])
    lo = getattr(a, "get", lambda k: None)
    print(tag, "ss", [float((a_ - b_).abs().max()) for a_, b_ in zip(a.get("_ss", []), b.get("_ss", []))])


net = fpm.Net(regression=True, backbone=False)
net.load_state_dict(sd)
ref = net(dd())
ref_out = dict(net.last_outputs)
ref2 = net(dd())
cmp("net-vs-net", ref, ref2)
sh = ShardedNet(net, devices=[0, 0])
out = sh(dd())
cmp("sharded-threads", ref, out)
print("sharded ss diff", float((sh.last_outputs["ss"].cpu() - ref_out["ss"].cpu()).abs().max()),
      "s diff", float((sh.last_outputs["s"].cpu() - ref_out["s"].cpu()).abs().max()))


class SyncThread:
    def __init__(self, target, args):
        self.t, self.a = target, args

    def start(self):
        self.t(*self.a)

    def join(self):
        pass


threading_Thread = threading.Thread
import fpm.parallel as FP  # noqa: E402
FP.threading.Thread = SyncThread
out2 = ShardedNet(net, devices=[0, 0])(dd())
cmp("sharded-serial", ref, out2)
FP.threading.Thread = threading_Thread
out3 = ShardedNet(net, devices=[0, 0])(dd(gt=False))
ref3 = net(dd(gt=False))
cmp("sharded-nogt", ref3, out3)
bt = net._batch_from_dict(dd(), torch.device("cuda", 0))
cmp("run-bt", net.run(bt), ShardedNet(net, devices=[0, 0]).run(bt))
