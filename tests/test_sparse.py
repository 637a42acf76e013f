"""API-parity sparse ops: fpm.sparse_torch / fpm.sparse / fpm.fgm.

CPU tests cover the containers, the host twins of the extension ops and the golden Kronecker
fixtures (generated from the reference's build_graphs / kronecker_sparse / CSCMatrix3d); GPU tests
compare the HIP kernels with the host twins and with dense products."""
import os

import numpy as np
import pytest
import scipy.sparse as ssp
import torch

import fpm
from fpm import fgm, sparse, sparse_torch as st
import oracle as O

from conftest import GOLDEN


def _rand_csr_list(B, h, w, density, seed, dtype=np.float32):
    rng = np.random.default_rng(seed)
    out = []
    for b in range(B):
        m = ssp.random(h, w, density=density, random_state=rng, dtype=np.float64).astype(dtype)
        out.append(m.tocsr())
    return out


def _dense(mats):
    return np.stack([m.toarray() for m in mats])


# ----------------------------------------------------------------------------------------------- CPU
def test_containers_roundtrip():
    mats = _rand_csr_list(3, 7, 5, 0.4, 0)
    a = st.CSRMatrix3d(mats)
    assert a.shape == (3, 7, 5) and len(a) == 3
    np.testing.assert_array_equal(a.numpy(), _dense(mats))
    np.testing.assert_array_equal(a[1].numpy()[0], mats[1].toarray())
    np.testing.assert_array_equal(a[0:3:2].numpy(), _dense(mats)[0::2])
    c = a.transpose()                           # CSR (b,h,w) -> CSC (b,w,h), same arrays
    assert isinstance(c, st.CSCMatrix3d) and c.shape == (3, 5, 7)
    np.testing.assert_array_equal(c.numpy(), _dense(mats).transpose(0, 2, 1))
    k = a.transpose(keep_type=True)
    assert isinstance(k, st.CSRMatrix3d)
    np.testing.assert_array_equal(k.numpy(), _dense(mats).transpose(0, 2, 1))
    cat = st.concatenate(a, a[0])
    np.testing.assert_array_equal(cat.numpy(), np.concatenate([_dense(mats), _dense(mats)[:1]]))
    d = torch.from_numpy(_dense(mats))
    np.testing.assert_array_equal(st.CSRMatrix3d.from_dense(d).numpy(), _dense(mats))
    np.testing.assert_array_equal(st.CSCMatrix3d.from_dense(d).numpy(), _dense(mats))
    sq = st.CSRMatrix3d(_rand_csr_list(2, 6, 6, 0.5, 1))
    np.testing.assert_array_equal(sq.diagonal().numpy(), np.stack([np.diag(m) for m in sq.numpy()]))
    assert torch.equal(sq.as_sparse_torch().to_dense(), torch.from_numpy(sq.numpy()))


def test_host_csr_dot_csc_and_diag():
    m1 = _rand_csr_list(2, 6, 9, 0.4, 2)
    m2 = _rand_csr_list(2, 9, 4, 0.4, 3)
    a = st.CSRMatrix3d(m1)
    b = st.CSCMatrix3d([m.tocsc() for m in m2])
    r = st.dot(a, b)
    assert isinstance(r, st.CSRMatrix3d)
    np.testing.assert_allclose(r.numpy(), _dense(m1) @ _dense(m2), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(a.dot(b, dense_output=True), _dense(m1) @ _dense(m2), rtol=1e-6, atol=1e-7)
    v = torch.rand(2, 9)
    dd = a.dotdiag(v)
    np.testing.assert_allclose(dd.numpy(), _dense(m1) * v.numpy()[:, None, :], rtol=1e-7)
    with pytest.raises(NotImplementedError):
        st.dot(torch.zeros(2, 6, 9), b, dense_output=True)     # dense x CSC on CPU: reference raises too


def test_host_bilinear_diag():
    m1 = _rand_csr_list(2, 5, 6, 0.5, 4, np.float64)
    m3 = _rand_csr_list(2, 6, 5, 0.5, 5, np.float64)
    s1 = st.CSRMatrix3d(m1)
    s3 = st.CSCMatrix3d([m.tocsc() for m in m3])
    d2 = torch.rand(2, 6, 6, dtype=torch.float64)
    out = sparse.bilinear_diag_torch(s1, d2, s3)
    ref = np.stack([np.diag(_dense(m1)[b] @ d2[b].numpy() @ _dense(m3)[b]) for b in range(2)])
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-12)


def test_kronecker_fixture_and_sparse_aff_mat():
    """Pinned against the reference's build_graphs + kronecker_sparse + CSCMatrix3d (collate,
    src/gmdataset.py:623-634) and construct_sparse_aff_mat outputs."""
    z = np.load(os.path.join(GOLDEN, "graphs_pattern.npz"))
    K1G = [fgm.kronecker_sparse(z["G2"], z["G1"]).astype(np.float32)]
    K1H = [fgm.kronecker_sparse(z["H2"], z["H1"]).astype(np.float32)]
    np.testing.assert_array_equal(st.CSCMatrix3d(K1G).indices.numpy(), z["kro_G"])
    np.testing.assert_array_equal(st.CSCMatrix3d(K1H).transpose().indices.numpy(), z["kro_H"])
    e1, e2 = z["G1"].shape[1], z["G2"].shape[1]
    Ke = torch.arange(e1 * e2, dtype=torch.float32).view(e1, e2) + 1000
    Kp = torch.arange(9 * 7, dtype=torch.float32).view(9, 7)
    val, row, col = fgm.construct_sparse_aff_mat(Ke, Kp, torch.from_numpy(z["kro_G"]).float(),
                                                 torch.from_numpy(z["kro_H"]).float())
    np.testing.assert_array_equal(val.numpy(), z["val"])
    np.testing.assert_array_equal(row.numpy(), z["row"])
    np.testing.assert_array_equal(col.numpy(), z["col"])
    G = torch.rand(2, 3, 4)
    H = torch.rand(2, 5, 2)
    kt = fgm.kronecker_torch(G, H)
    for b in range(2):
        np.testing.assert_allclose(kt[b].numpy(), np.kron(G[b].numpy(), H[b].numpy()), rtol=1e-6)


def _fgm_inputs(z):
    K1G = [fgm.kronecker_sparse(z["G2"], z["G1"]).astype(np.float32)]
    K1H = [fgm.kronecker_sparse(z["H2"], z["H1"]).astype(np.float32)]
    return st.CSRMatrix3d(K1G), st.CSRMatrix3d(K1H).transpose()       # the KGHs pair (gmdataset.py:648-650)


def _edges(G, H):
    return torch.stack([torch.from_numpy(G.argmax(0)), torch.from_numpy(H.argmax(0))])


def test_dense_fgm_matches_factorized_pattern():
    """Cross-check of a6/a7: the dense FGM rebuild (RebuildFGM.forward) with Ke = 1, Kp = 1 counts
    exactly the Kronecker edge pairs + diagonal that the index-free GNN aggregation assumes."""
    z = np.load(os.path.join(GOLDEN, "graphs_pattern.npz"))
    KG, KH = _fgm_inputs(z)
    e1, e2 = z["G1"].shape[1], z["G2"].shape[1]
    n1, n2 = z["G1"].shape[0], z["G2"].shape[0]
    K = fgm.construct_aff_mat(torch.ones(1, e1, e2), torch.ones(1, n1, n2), KG, KH)[0]
    row, col = O.kron_pattern(_edges(z["G1"], z["H1"]), _edges(z["G2"], z["H2"]), n1, n2, n1, n2)
    cnt = torch.zeros(n1 * n2, n1 * n2)
    cnt.index_put_((row, col), torch.ones(row.numel()), accumulate=True)
    assert torch.equal(K, cnt)
    # generic values: K = diag(vec Kp) + kron(G2,G1) diag(vec Ke) kron(H2,H1)^T  (column-major vecs)
    g = torch.Generator().manual_seed(0)
    Ke = torch.rand(1, e1, e2, generator=g, dtype=torch.float64)
    Kp = torch.rand(1, n1, n2, generator=g, dtype=torch.float64)
    KG64, KH64 = KG.to(torch.float64), KH.to(torch.float64)
    K = fgm.construct_aff_mat(Ke, Kp, KG64, KH64)[0].numpy()
    kg = np.kron(z["G2"], z["G1"]).astype(np.float64)
    kh = np.kron(z["H2"], z["H1"]).astype(np.float64)
    ref = np.diag(Kp[0].t().reshape(-1).numpy()) + kg @ np.diag(Ke[0].t().reshape(-1).numpy()) @ kh.T
    np.testing.assert_allclose(K, ref, rtol=1e-12, atol=1e-12)


# ----------------------------------------------------------------------------------------------- GPU
DEV = torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.float16])
def test_device_products_vs_host(dt):
    m1 = _rand_csr_list(3, 40, 700, 0.05, 10)       # rows longer than one LDS pass in places
    m2 = _rand_csr_list(3, 700, 33, 0.05, 11)
    a = st.CSRMatrix3d(m1).to(dt)
    b = st.CSCMatrix3d([m.tocsc() for m in m2]).to(dt)
    ref = torch.from_numpy(_dense(m1)).double() @ torch.from_numpy(_dense(m2)).double()
    tol = {torch.float32: 1e-5, torch.float64: 1e-12, torch.float16: 5e-2}[dt]
    out = st.dot(a.cuda(), b.cuda(), dense_output=True).cpu().double()
    assert (out - ref).abs().max() < tol * max(1.0, ref.abs().max())
    d1 = torch.from_numpy(_dense(m1)).to(dt).to(DEV)
    out2 = st.dot(d1, b.cuda(), dense_output=True).cpu().double()
    assert (out2 - ref).abs().max() < tol * max(1.0, ref.abs().max())
    if dt != torch.float16:
        host = st.dot(a, b, dense_output=True)
        assert np.abs(out.numpy() - host).max() <= tol * max(1.0, float(ref.abs().max()))
    v = torch.rand(3, 700).to(dt)
    dd = a.cuda().dotdiag(v.to(DEV))
    ref_dd = a.dotdiag(v) if dt != torch.float16 else None
    if ref_dd is not None:
        assert torch.equal(dd.data.cpu(), ref_dd.data)
    assert torch.equal(dd.indices.cpu(), a.indices) and torch.equal(dd.indptr.cpu(), a.indptr)


@pytest.mark.gpu
def test_device_bilinear_diag_and_fgm_backward():
    z = np.load(os.path.join(GOLDEN, "graphs_pattern.npz"))
    KG, KH = _fgm_inputs(z)
    KG, KH = KG.to(torch.float64).cuda(), KH.to(torch.float64).cuda()
    e1, e2 = z["G1"].shape[1], z["G2"].shape[1]
    n1, n2 = z["G1"].shape[0], z["G2"].shape[0]
    g = torch.Generator().manual_seed(1)
    Ke = torch.rand(1, e1, e2, generator=g, dtype=torch.float64).to(DEV).requires_grad_()
    Kp = torch.rand(1, n1, n2, generator=g, dtype=torch.float64).to(DEV).requires_grad_()
    K = fgm.construct_aff_mat(Ke, Kp, KG, KH)
    kg = np.kron(z["G2"], z["G1"]).astype(np.float64)
    kh = np.kron(z["H2"], z["H1"]).astype(np.float64)
    ref = np.diag(Kp[0].detach().t().reshape(-1).cpu().numpy()) + \
        kg @ np.diag(Ke[0].detach().t().reshape(-1).cpu().numpy()) @ kh.T
    np.testing.assert_allclose(K[0].detach().cpu().numpy(), ref, rtol=1e-12, atol=1e-12)
    W = torch.rand(K.shape, generator=g, dtype=torch.float64).to(DEV)
    (K * W).sum().backward()
    Wn = W[0].cpu().numpy()
    dKe_ref = np.einsum("pe,pq,qe->e", kg, Wn, kh).reshape(e2, e1).T     # vec is column-major
    np.testing.assert_allclose(Ke.grad[0].cpu().numpy(), dKe_ref, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(Kp.grad[0].cpu().numpy(), np.diag(Wn).reshape(n2, n1).T, rtol=0, atol=0)
