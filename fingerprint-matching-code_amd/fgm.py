"""Factorized graph matching helpers (utils/factorize_graph_matching.py) on the fpm sparse ops.

* ``construct_aff_mat(Ke, Kp, KroG, KroH)`` -> dense K = diag(vec Kp) + (G2 (x) G1) diag(vec Ke)
  (H2 (x) H1)^T via ``RebuildFGM`` (forward :151-166 = CSR.dotdiag then CSR x CSC -> dense;
  backward :168-186 = bilinear_diag for dKe, diagonal for dKp).
* ``construct_sparse_aff_mat`` (:57-95), ``kronecker_torch`` (:98-122), ``kronecker_sparse``
  (:125-137).
Off the live forward (ngm.py:293-315 is commented out); the live path uses the index-free
factorized aggregation of csrc/gnn.hip.  These give API parity and the small-n dense cross-check.
"""
import scipy.sparse as ssp
import torch
from torch.autograd import Function

from .sparse import bilinear_diag_torch
from .sparse_torch import CSRMatrix3d, CSCMatrix3d


class RebuildFGM(Function):
    @staticmethod
    def forward(ctx, Ke, Kp, Kro1, Kro2, Kro1T=None, Kro2T=None):
        ctx.save_for_backward(Ke, Kp)
        if Kro1T is not None and Kro2T is not None:
            ctx.K = Kro1T, Kro2T
        else:
            ctx.K = Kro1.transpose(keep_type=True), Kro2.transpose(keep_type=True)
        B = Ke.shape[0]
        kro1ke = Kro1.dotdiag(Ke.transpose(1, 2).contiguous().view(B, -1))
        K = kro1ke.dot(Kro2, dense_output=True)
        K = torch.as_tensor(K, device=Ke.device)
        diag = Kp.transpose(1, 2).contiguous().view(B, -1)
        return K + torch.diag_embed(diag).to(K.dtype)

    @staticmethod
    def backward(ctx, dK):
        Ke, Kp = ctx.saved_tensors
        k1t, k2t = ctx.K
        dKe = dKp = None
        if ctx.needs_input_grad[0]:
            dKe = bilinear_diag_torch(k1t, dK.contiguous(), k2t)
            dKe = dKe.view(Ke.shape[0], Ke.shape[2], Ke.shape[1]).transpose(1, 2)
        if ctx.needs_input_grad[1]:
            dKp = torch.diagonal(dK, dim1=-2, dim2=-1)
            dKp = dKp.reshape(Kp.shape[0], Kp.shape[2], Kp.shape[1]).transpose(1, 2)
        return dKe, dKp, None, None, None, None


def construct_aff_mat(Ke, Kp, KroG: CSRMatrix3d, KroH: CSCMatrix3d, KroGt=None, KroHt=None):
    return RebuildFGM.apply(Ke, Kp, KroG, KroH, KroGt, KroHt)


def construct_sparse_aff_mat(Ke, Kp, row_idx, col_idx):
    """Values then indices of K's nonzeros: Ke's entries followed by the n1n2 diagonal (float
    indices from linspace, as the reference)."""
    ev = torch.flatten(Ke)
    pv = torch.flatten(Kp)
    n = pv.shape[0]
    diag = torch.linspace(0, n - 1, n, device=row_idx.device)
    return torch.cat((ev, pv), 0), torch.cat((row_idx, diag), 0), torch.cat((col_idx, diag), 0)


def kronecker_torch(t1, t2):
    B = t1.shape[0]
    a1, a2 = t1.shape[1], t1.shape[2]
    b1, b2 = t2.shape[1], t2.shape[2]
    tt = torch.bmm(t1.reshape(B, -1, 1), t2.reshape(B, 1, -1))
    return tt.reshape(B, a1, a2, b1, b2).permute(0, 1, 3, 2, 4).reshape(B, a1 * b1, a2 * b2)


def kronecker_sparse(arr1, arr2):
    return ssp.kron(ssp.coo_matrix(arr1), ssp.coo_matrix(arr2))
