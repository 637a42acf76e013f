"""Streaming Sinkhorn, split vs one-workgroup form: per-pair max error vs the fp64 oracle and their
difference (both layouts, tau 0.01 / 0.0005).   python tools/sk_split_diag.py"""
import sys, os, torch
sys.path.insert(0, os.getcwd())
from fpm import ops, _lib
import oracle as O
DEV = torch.device("cuda", 0)
def i32(v): return torch.tensor(v, dtype=torch.int32, device=DEV)
g = torch.Generator().manual_seed(31)
n1s, n2s = (512, 400, 300, 512, 260, 256, 512), (512, 400, 512, 300, 260, 256, 497)
B = len(n1s)
s = torch.randn(B, 512, 512, generator=g) * 0.3
for tau in (0.01, 0.0005):
    ref = O.pygm_sinkhorn(s.double(), n1s, n2s, dummy_row=True, max_iter=10, tau=tau)
    sd = s.to(DEV); n1d, n2d = i32(n1s), i32(n2s)
    out = ops.sinkhorn(sd, n1d, n2d, 10, tau, True)
    one = torch.empty_like(out)
    _lib.call("fpm_sinkhorn_log_fwd", ops._p(sd), *sd.stride(), ops._p(one), *one.stride(), ops._p(n1d), ops._p(n2d), B, 512, 512, 10, float(tau), 1, ops._stream(sd))
    sT = s.transpose(1, 2).contiguous().to(DEV).transpose(1, 2)
    o2 = torch.zeros(B, 512, 512, device=DEV).transpose(1, 2)
    ops.sinkhorn(sT, n1d, n2d, 10, tau, True, out=o2)
    o3 = torch.zeros(B, 512, 512, device=DEV).transpose(1, 2)
    _lib.call("fpm_sinkhorn_log_fwd", ops._p(sT), *sT.stride(), ops._p(o3), *o3.stride(), ops._p(n1d), ops._p(n2d), B, 512, 512, 10, float(tau), 1, ops._stream(sd))
    torch.cuda.synchronize()
    for name, t in (("split", out), ("one", one), ("splitT", o2), ("oneT", o3)):
        e = (t.cpu().double() - ref).abs().amax(dim=(1, 2))
        print(tau, name, ["%.2e" % x for x in e.tolist()])
    print(tau, "split - one", ["%.2e" % x for x in (out - one).abs().amax(dim=(1, 2)).tolist()],
          "T", ["%.2e" % x for x in (o2 - o3).abs().amax(dim=(1, 2)).tolist()])
