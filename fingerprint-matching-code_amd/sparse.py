"""``bilinear_diag_torch`` (src/sparse.py:182-235): diag(S1 . D2 . S3) per batch, S1 CSR (b, x, y),
D2 dense (b, y, y), S3 CSC (b, y, x) -> (b, x).  Device tensors run the HIP kernel
``fpm_bilinear_diag``; CPU tensors its host twin (the reference runs both, bilinear_diag.cpp:303-320)."""
import ctypes

import torch

from . import _lib
from .sparse_torch import CSRMatrix3d, CSCMatrix3d, _code, _p, _same_device, _stream


def bilinear_diag_torch(s_t1: CSRMatrix3d, d_t2: torch.Tensor, s_t3: CSCMatrix3d, device=None):
    if device is None:
        device = d_t2.device
    B, xlen = s_t1.shape[0], s_t1.shape[1]
    assert s_t1.shape[0] == d_t2.shape[0] == s_t3.shape[0], 'Batch size mismatch.'
    assert s_t1.shape[1] == s_t3.shape[2], 'Sparse matrix 1 & 3 shape mismatch.'
    assert s_t1.shape[2] == d_t2.shape[1] == d_t2.shape[2] == s_t3.shape[1], 'Matrix size mismatch.'
    t2 = d_t2.contiguous()
    d1 = s_t1.data.to(t2.dtype).contiguous()
    d3 = s_t3.data.to(t2.dtype).contiguous()
    _same_device(t2.device, s_t1.indices, s_t1.indptr, d1, s_t3.indices, s_t3.indptr, d3)
    out = torch.empty(B, xlen, dtype=t2.dtype, device=t2.device)
    args = (_p(s_t1.indices), _p(s_t1.indptr), _p(d1), _p(t2), t2.shape[1], _p(s_t3.indices), _p(s_t3.indptr),
            _p(d3), B, xlen, _p(out))
    if t2.is_cuda:
        _lib.call("fpm_bilinear_diag", _code(t2), *args, _stream(t2.device))
    else:
        _lib.call("fpm_bilinear_diag_host", _code(t2, True), *args)
    return out.to(device)
