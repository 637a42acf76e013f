"""``Gconv`` / ``Siamese_Gconv`` (src/model/gcn.py:8-38, 118-141) over ``fpm_gconv_fwd``.

Same module surface (a_fc / u_fc Linear parameters, forward(A, x, norm=True)); the forward runs
the HIP kernels and raises on CPU tensors (no CPU fallback)."""
import ctypes

import torch
import torch.nn as nn

from . import _lib


class Gconv(nn.Module):
    def __init__(self, in_features, out_features):
        super().__init__()
        self.num_inputs = in_features
        self.num_outputs = out_features
        self.a_fc = nn.Linear(in_features, out_features)
        self.u_fc = nn.Linear(in_features, out_features)

    def forward(self, A, x, norm=True):
        if not (A.is_cuda and x.is_cuda):
            raise _lib.FpmError("Gconv: the HIP path has no CPU fallback")
        B, n, din = x.shape
        dout = self.num_outputs
        A = A.float().contiguous()
        x = x.float().contiguous()
        dev = x.device
        if A.device != dev:
            raise _lib.FpmError("Gconv: A and x must be on the same device")
        W = torch.cat([self.a_fc.weight, self.u_fc.weight]).detach().to(dev, torch.float32).contiguous()
        b = torch.cat([self.a_fc.bias, self.u_fc.bias]).detach().to(dev, torch.float32).contiguous()
        if tuple(A.shape) != (B, n, n) or W.shape[1] != din:
            raise _lib.FpmError("Gconv: shape mismatch A %s x %s" % (tuple(A.shape), tuple(x.shape)))
        ws = torch.empty(_lib.load().fpm_gconv_ws_floats(B, n, dout), device=x.device, dtype=torch.float32)
        out = torch.empty(B, n, dout, device=x.device, dtype=torch.float32)
        st = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        _lib.call("fpm_gconv_fwd", p(A), p(x), B, n, din, dout, p(W), p(b), int(bool(norm)), p(ws), p(out), st)
        return out


class Siamese_Gconv(nn.Module):
    def __init__(self, in_features, num_features):
        super().__init__()
        self.gconv = Gconv(in_features, num_features)

    def forward(self, g1, *args):
        emb1 = self.gconv(*g1)
        if len(args) == 0:
            return emb1
        return [emb1] + [self.gconv(*g) for g in args]
