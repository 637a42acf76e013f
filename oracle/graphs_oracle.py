"""CPU restatement of the reference's graph construction — TEST ORACLE ONLY (see ``oracle/__init__``).

Restates ``utils/build_graphs.py:12-120`` (build_graphs with 'tri' / 'fc' / 'near', sym=True,
delaunay_triangulate over scipy.spatial.Delaunay, fully_connect), ``GMDataset.to_pyg_graph``
(``src/gmdataset.py:170-189``: edge_index = np.nonzero(A), edge_attr = clip(0.5*(P_i-P_j)/320+0.5))
and the collate's Kronecker index lists (``src/gmdataset.py:623-634`` over
``utils/factorize_graph_matching.py:125-137`` kronecker_sparse and ``CSCMatrix3d.indices``).
Pinned by ``tests/golden/delaunay.npz`` and ``tests/golden/graphs_pattern.npz`` (generated from the
reference's own build_graphs / kronecker_sparse / CSCMatrix3d).
"""
import numpy as np
import scipy.sparse as ssp
from scipy.spatial import Delaunay

PSEUDO_RESCALE = 320.0  # max(RESCALE), gmdataset.py:36,171


def fully_connect(P, thre=None):
    """build_graphs.py:103-119."""
    n = P.shape[0]
    A = np.ones((n, n)) - np.eye(n)
    if thre is not None:
        for i in range(n):
            for j in range(i):
                if np.linalg.norm(P[i] - P[j]) > thre:
                    A[i, j] = 0
                    A[j, i] = 0
    return A


def delaunay_triangulate(P):
    """build_graphs.py:77-100 (scipy Delaunay simplices -> symmetric adjacency; QhullError -> fc)."""
    n = P.shape[0]
    if n < 3:
        return fully_connect(P)
    try:
        d = Delaunay(P)
    except Exception:  # scipy.spatial.QhullError (flat input)
        return fully_connect(P)
    A = np.zeros((n, n))
    s = d.simplices
    for a, b in ((0, 1), (0, 2), (1, 2)):
        A[s[:, a], s[:, b]] = 1
        A[s[:, b], s[:, a]] = 1
    return A


def build_graphs(P, n, n_pad=None, edge_pad=None, stg="fc", sym=True, thre=0):
    """build_graphs.py:12-74 -> (A, G, H, edge_num)."""
    assert stg in ("fc", "tri", "near")
    if stg == "tri":
        A = delaunay_triangulate(P[0:n, :])
    elif stg == "near":
        A = fully_connect(P[0:n, :], thre=thre)
    else:
        A = fully_connect(P[0:n, :])
    edge_num = int(np.sum(A, axis=(0, 1)))
    n_pad = n if n_pad is None else n_pad
    edge_pad = edge_num if edge_pad is None else edge_pad
    G = np.zeros((n_pad, edge_pad), dtype=np.float32)
    H = np.zeros((n_pad, edge_pad), dtype=np.float32)
    src, dst = np.nonzero(A) if sym else np.nonzero(np.triu(A))
    G[src, np.arange(src.size)] = 1
    H[dst, np.arange(dst.size)] = 1
    return A, G, H, edge_num


def pyg_edges(A, P, rescale=PSEUDO_RESCALE):
    """GMDataset.to_pyg_graph (gmdataset.py:170-176): edge_index (2, E) int64, edge_attr (E, 2) fp32."""
    P = np.asarray(P, dtype=np.float64)
    edge_feat = 0.5 * (np.expand_dims(P, axis=1) - np.expand_dims(P, axis=0)) / rescale + 0.5
    ei = np.nonzero(A)
    attr = np.clip(edge_feat[ei], 0, 1).astype(np.float32)
    return np.stack(ei).astype(np.int64), attr


def kron_pattern(G1, H1, G2, H2):
    """Collate Kronecker index lists of one pair (gmdataset.py:623-634): CSC row indices of
    kron(G2, G1) and the CSC(kron(H2, H1)).transpose() indices, both in column (edge-pair) order."""
    kg = ssp.kron(ssp.coo_matrix(G2), ssp.coo_matrix(G1)).tocsc()
    kh = ssp.kron(ssp.coo_matrix(H2), ssp.coo_matrix(H1)).tocsc()
    kg.sort_indices()
    kh.sort_indices()
    return kg.indices.astype(np.int64), kh.indices.astype(np.int64)
