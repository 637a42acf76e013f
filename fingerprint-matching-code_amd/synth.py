"""Synthetic keypoint-graph pairs for the benchmark configs (host-side input preparation).

Each pair p and side g draws from its own seeded stream (``hash(base_seed, p, g)``):
  * n keypoints ~ U([0,320) x [0,240))  (image frame of ``src/gmdataset.py:17-32``);
  * Delaunay adjacency, symmetric, as ``utils/build_graphs.py:77-100`` ('tri', sym=True);
  * directed edge list = ``np.nonzero(A)`` (row-major), pseudo-coordinates
    ``clip(0.5*(P_src-P_dst)/320 + 0.5, 0, 1)`` (``GMDataset.to_pyg_graph``, gmdataset.py:170-189);
  * node features = [L2norm(N(0,1)^256) || L2norm(N(0,1)^512)] per keypoint
    (mimics ``normalize_over_channels`` + ``feature_align``, ngm.py:241-248);
  * global feature = |N(0,1)|^512 (post-ReLU pooled map, ngm.py:238).
Graph construction is input preparation (the reference does it in DataLoader workers) and is
not part of the timed forward.
"""
import numpy as np
from scipy.spatial import Delaunay

from . import config as C


def _rng(base_seed, p, g):
    return np.random.default_rng(np.random.SeedSequence([int(base_seed), int(p), int(g)]))


def delaunay_adjacency(P):
    """Symmetric 0/1 adjacency of the Delaunay triangulation (build_graphs.py:77-100)."""
    n = P.shape[0]
    if n < 3:
        A = np.ones((n, n)) - np.eye(n)
        return A
    d = Delaunay(P)
    A = np.zeros((n, n))
    s = d.simplices
    for a, b in ((0, 1), (0, 2), (1, 2)):
        A[s[:, a], s[:, b]] = 1
        A[s[:, b], s[:, a]] = 1
    return A


def edges_from_adjacency(A, P):
    """(edge_index (2,E) int64, pseudo (E,2) float32) as GMDataset.to_pyg_graph builds them."""
    src, dst = np.nonzero(A)
    pseudo = 0.5 * (P[src] - P[dst]) / C.PSEUDO_RESCALE + 0.5
    pseudo = np.clip(pseudo, 0, 1).astype(np.float32)
    return np.stack([src, dst]).astype(np.int64), pseudo


def make_graph(base_seed, p, g, n):
    rng = _rng(base_seed, p, g)
    while True:
        # keypoints are float32 (the reference's Ps tensors); graphs are built from those values
        P = np.stack([rng.uniform(0, 320, n), rng.uniform(0, 240, n)], axis=1).astype(np.float32).astype(np.float64)
        if len(np.unique(P, axis=0)) == n:
            break
    A = delaunay_adjacency(P)
    ei, pseudo = edges_from_adjacency(A, P)
    x = rng.standard_normal((n, C.NODE_FEATURE_DIM)).astype(np.float32)
    a = C.FEATURE_CHANNEL_NODE
    x[:, :a] /= np.linalg.norm(x[:, :a], axis=1, keepdims=True)
    x[:, a:] /= np.linalg.norm(x[:, a:], axis=1, keepdims=True)
    w = np.abs(rng.standard_normal(C.GLOBAL_FEATURE_DIM)).astype(np.float32)
    return dict(P=P.astype(np.float32), A=A.astype(np.float32), edge_index=ei, pseudo=pseudo,
                x=x, w=w, n=n)


def make_batch(base_seed, B, n1, n2=None, first_pair=0):
    """List of B pairs, each a tuple (graph_side0, graph_side1).

    ``n1``/``n2`` are ints or per-pair sequences (ragged batches)."""
    n2 = n1 if n2 is None else n2
    pairs = []
    for b in range(B):
        p = first_pair + b
        na = n1[b] if hasattr(n1, "__len__") else n1
        nb = n2[b] if hasattr(n2, "__len__") else n2
        pairs.append((make_graph(base_seed, p, 0, na), make_graph(base_seed, p, 1, nb)))
    return pairs
