"""On-device graph construction (fpm.graphs, csrc/graphs.hip) vs the CPU oracle
(oracle/graphs_oracle.py = utils/build_graphs.py + GMDataset.to_pyg_graph + the collate's
Kronecker index lists, pinned by the reference-generated fixtures delaunay.npz / graphs_pattern.npz).

Bar: identical adjacency, edge order, incidence matrices and Kronecker index lists (integer work),
bit-identical pseudo-coordinates (same fp64 expression rounded to fp32).  Delaunay is compared on
random keypoints in general position (uniform floats in the 320x240 frame); four exactly
cocircular points are a documented non-goal (Qhull's 'Qt' picks a diagonal arbitrarily).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import graphs_oracle as GO


def _points(rng, n):
    while True:
        P = np.stack([rng.uniform(0, 320, n), rng.uniform(0, 240, n)], 1).astype(np.float32)
        if len(np.unique(P, axis=0)) == n:
            return P


# ------------------------------------------------------------------------------- CPU: oracle pins
def test_oracle_build_graphs_golden():
    z = np.load(os.path.join(GOLDEN, "delaunay.npz"))
    for c in range(int(z["ncases"])):
        P = z["c%d_P" % c].astype(np.float64)
        A, G, H, e = GO.build_graphs(P, len(P), stg="tri")
        assert np.array_equal(A, z["c%d_A" % c])
        assert np.array_equal(G, z["c%d_G" % c]) and np.array_equal(H, z["c%d_H" % c])


def test_oracle_kron_pattern_golden():
    z = np.load(os.path.join(GOLDEN, "graphs_pattern.npz"))
    A1, G1, H1, _ = GO.build_graphs(z["P1"], 9, stg="tri")
    A2, G2, H2, _ = GO.build_graphs(z["P2"], 7, stg="tri")
    for a, b in ((A1, "A1"), (G1, "G1"), (H1, "H1"), (A2, "A2"), (G2, "G2"), (H2, "H2")):
        assert np.array_equal(a, z[b]), b
    kg, kh = GO.kron_pattern(G1, H1, G2, H2)
    assert np.array_equal(kg, z["kro_G"]) and np.array_equal(kh, z["kro_H"])


# ------------------------------------------------------------------------------- GPU
DEV = torch.device("cuda", 0)


def _batch(Ps, nmax):
    P = np.zeros((len(Ps), nmax, 2), np.float32)
    for g, p in enumerate(Ps):
        P[g, :len(p)] = p
    return torch.from_numpy(P).to(DEV), [len(p) for p in Ps]


def _check_batch(Ps, stg="tri", thre=0.0):
    from fpm import graphs
    nmax = max(len(p) for p in Ps)
    P, ns = _batch(Ps, nmax)
    gb = graphs.build_graph_batch(P, ns, stg=stg, thre=thre, want_A=True)
    A = gb.A.cpu().numpy()
    src, dst, pseudo = gb.src.cpu().numpy(), gb.dst.cpu().numpy(), gb.pseudo.cpu().numpy()
    off = gb.edge_off.cpu().numpy()
    assert np.array_equal(off, gb.edge_off_host.numpy())
    for g, p in enumerate(Ps):
        n = len(p)
        Pd = p.astype(np.float64)
        if stg == "tri":
            Ar = GO.delaunay_triangulate(Pd)
        else:
            Ar = GO.fully_connect(Pd, thre=thre if stg == "near" else None)
        assert np.array_equal(A[g, :n, :n], Ar), (g, n, np.argwhere(A[g, :n, :n] != Ar)[:5])
        assert not A[g, n:].any() and not A[g, :, n:].any()
        ei, attr = GO.pyg_edges(Ar, Pd)
        e0, e1 = off[g], off[g + 1]
        assert np.array_equal(src[e0:e1] - g * nmax, ei[0])
        assert np.array_equal(dst[e0:e1] - g * nmax, ei[1])
        assert np.array_equal(pseudo[e0:e1], attr)
    return gb


@pytest.mark.gpu
@pytest.mark.parametrize("n,count", [(3, 64), (4, 64), (7, 64), (12, 64), (40, 64), (128, 32), (256, 32),
                                     (512, 8), (1024, 2)])
def test_delaunay_vs_scipy(n, count):
    rng = np.random.default_rng(1000 + n)
    _check_batch([_points(rng, n) for _ in range(count)])


@pytest.mark.gpu
def test_delaunay_ragged_batch():
    rng = np.random.default_rng(5)
    ns = [1, 2, 3, 5, 33, 64, 100, 129, 200, 256, 17, 250]
    _check_batch([_points(rng, n) for n in ns])


@pytest.mark.gpu
def test_delaunay_degenerate_inputs():
    """Flat inputs raise QhullError in the reference -> fully connected (build_graphs.py:96-100);
    collinear hull points: the middle point splits the hull edge."""
    line = np.stack([np.linspace(0, 300, 9), np.linspace(10, 100, 9)], 1).astype(np.float32)
    line2 = np.stack([np.arange(6) * 16.0, np.full(6, 40.0)], 1).astype(np.float32)
    # a square grid corner row: three collinear points on the hull bottom plus interior points
    rng = np.random.default_rng(9)
    hull = np.concatenate([np.array([[0, 0], [100, 0], [200, 0]], np.float32),
                           np.stack([rng.uniform(5, 195, 20), rng.uniform(5, 150, 20)], 1).astype(np.float32)])
    _check_batch([line, line2, hull])


@pytest.mark.gpu
def test_fc_and_near():
    rng = np.random.default_rng(11)
    Ps = [_points(rng, n) for n in (2, 9, 31, 70)]
    _check_batch(Ps, stg="fc")
    _check_batch(Ps, stg="near", thre=80.0)


@pytest.mark.gpu
def test_build_graphs_golden():
    """fpm.graphs.build_graphs (A, G, H, edge_num) == the reference's build_graphs fixtures."""
    from fpm import graphs
    z = np.load(os.path.join(GOLDEN, "delaunay.npz"))
    for c in range(int(z["ncases"])):
        P = z["c%d_P" % c]
        A, G, H, e = graphs.build_graphs(torch.from_numpy(P), len(P), stg="tri")
        assert np.array_equal(A.cpu().numpy(), z["c%d_A" % c])
        assert np.array_equal(G.cpu().numpy(), z["c%d_G" % c])
        assert np.array_equal(H.cpu().numpy(), z["c%d_H" % c])
        assert e == int(z["c%d_A" % c].sum())
    # padded form
    P = z["c0_P"]
    A, G, H, e = graphs.build_graphs(torch.from_numpy(P), len(P), n_pad=20, edge_pad=70, stg="tri")
    Ar, Gr, Hr, er = GO.build_graphs(P.astype(np.float64), len(P), n_pad=20, edge_pad=70, stg="tri")
    assert np.array_equal(G.cpu().numpy(), Gr) and np.array_equal(H.cpu().numpy(), Hr) and e == er


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.int64])
def test_kronecker_pattern_golden(dtype):
    """Collate KGHs_sparse index lists (gmdataset.py:623-634) from the device edge lists."""
    from fpm import graphs
    z = np.load(os.path.join(GOLDEN, "graphs_pattern.npz"))
    P1 = torch.from_numpy(z["P1"].astype(np.float32))
    P2 = torch.from_numpy(z["P2"].astype(np.float32))
    g1 = graphs.build_graph_batch(P1.reshape(1, 9, 2).to(DEV), [9])
    g2 = graphs.build_graph_batch(P2.reshape(1, 7, 2).to(DEV), [7])
    rowG, colH = graphs.kronecker_pattern(g1.src, g1.dst, g2.src, g2.dst, n1pad=9, dtype=dtype)
    assert np.array_equal(rowG.cpu().numpy().astype(np.int64), z["kro_G"])
    assert np.array_equal(colH.cpu().numpy().astype(np.int64), z["kro_H"])


@pytest.mark.gpu
def test_kronecker_pattern_batch_vs_oracle():
    """Pairs inside a batch (batch-global node ids, padded n1) vs scipy kron over the oracle's G/H."""
    from fpm import graphs
    rng = np.random.default_rng(21)
    Ps1 = [_points(rng, n) for n in (12, 30, 25)]
    Ps2 = [_points(rng, n) for n in (14, 22, 30)]
    P1, n1 = _batch(Ps1, 30)
    P2, n2 = _batch(Ps2, 30)
    g1 = graphs.build_graph_batch(P1, n1)
    g2 = graphs.build_graph_batch(P2, n2)
    o1, o2 = g1.edge_off_host, g2.edge_off_host
    for b in range(3):
        a1, G1, H1, _ = GO.build_graphs(Ps1[b].astype(np.float64), n1[b], n_pad=30, stg="tri")
        a2, G2, H2, _ = GO.build_graphs(Ps2[b].astype(np.float64), n2[b], n_pad=30, stg="tri")
        kg, kh = GO.kron_pattern(G1, H1, G2, H2)
        s1, d1 = g1.src[o1[b]:o1[b + 1]], g1.dst[o1[b]:o1[b + 1]]
        s2, d2 = g2.src[o2[b]:o2[b + 1]], g2.dst[o2[b]:o2[b + 1]]
        rowG, colH = graphs.kronecker_pattern(s1, d1, s2, d2, n1pad=30, base1=b * 30, base2=b * 30,
                                              dtype=torch.int64)
        assert np.array_equal(rowG.cpu().numpy(), kg) and np.array_equal(colH.cpu().numpy(), kh)


@pytest.mark.gpu
def test_forward_from_keypoints_equals_host_graphs():
    """Keypoints -> device graphs -> forward is bit-identical to the forward over host-built graphs."""
    import fpm
    from fpm import params, synth
    from fpm.batch import DeviceBatch
    sd = params.init_params(3)
    rng = np.random.default_rng(31)
    B, ns1, ns2 = 5, [48, 40, 48, 33, 48], [48, 48, 41, 48, 30]
    pairs, P = [], [np.zeros((B, 48, 2), np.float32), np.zeros((B, 48, 2), np.float32)]
    for b in range(B):
        pr = []
        for side, n in ((0, ns1[b]), (1, ns2[b])):
            g = synth.make_graph(77, b, side, n)
            p32 = g["P"].astype(np.float32)
            A = GO.delaunay_triangulate(p32.astype(np.float64))
            ei, attr = GO.pyg_edges(A, p32)
            g = dict(g, A=A.astype(np.float32), edge_index=ei, pseudo=attr)
            P[side][b, :n] = p32
            pr.append(g)
        pairs.append(tuple(pr))
    net = fpm.Net(regression=True, backbone=False)
    net.load_state_dict(sd)
    host = DeviceBatch.from_pairs(pairs, DEV)
    dev = DeviceBatch.from_keypoints([torch.from_numpy(P[0]).to(DEV), torch.from_numpy(P[1]).to(DEV)],
                                     [ns1, ns2], host.x, host.w, DEV)
    for side in range(2):
        assert torch.equal(dev.src[side], host.src[side]) and torch.equal(dev.dst[side], host.dst[side])
        assert torch.equal(dev.pseudo[side], host.pseudo[side])
    a = net.run(host)
    b = net.run(dev, chunks=2)
    c = net.run(host, chunks=2)
    for k in ("ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert torch.equal(b[k], c[k]), k
        assert torch.equal(a[k], c[k]), k
