"""On-device keypoint-graph construction over the C-ABI (``fpm_graph_*``).

Mirrors the reference's DataLoader-side graph code so a GPU pipeline can go from keypoints to the
matcher's inputs without a host round trip:

* ``build_graphs(P, n, n_pad, edge_pad, stg, sym, thre)`` — ``utils/build_graphs.py:12-74``
  (A, G, H, edge_num) for one graph, as device tensors;
* ``build_graph_batch(P, n, stg, thre)`` — the same for G graphs at once (padded (G, nmax, 2)
  keypoints), returning the edge lists ``GMDataset.to_pyg_graph`` builds (src/gmdataset.py:170-189:
  edge_index = np.nonzero(A) row-major, edge_attr = clip(0.5*(P_src-P_dst)/320 + 0.5, 0, 1)) with
  batch-global node ids, plus per-graph edge offsets;
* ``kronecker_pattern(...)`` — the collate's ``KGHs_sparse`` index lists of one pair
  (src/gmdataset.py:623-634).

Delaunay ('tri') is an exact-predicate empty-circle test per candidate edge (``csrc/graphs.hip``);
for points in general position it equals scipy's Qhull triangulation.  Like the reference, n < 3
and all-collinear inputs give the fully connected graph.  Only ``sym=True`` (the reference's
SYM_ADJACENCY, gmdataset.py:39) is supported.
"""
import torch

from . import _lib
from . import config as C
from .ops import _dev, _p, _stream

STRATEGIES = {"tri": 0, "fc": 1, "near": 2}


def _check(rc):
    if rc != 0:
        raise _lib.FpmError(_lib.load().fpm_last_error().decode())


class GraphBatch:
    """Device result of ``build_graph_batch``: adjacency bits, degrees, edges, offsets."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def build_graph_batch(P, n, stg="tri", thre=0.0, want_A=False, want_GH=False, epad=None,
                      rescale=C.PSEUDO_RESCALE):
    """P: (G, nmax, 2) fp32 device keypoints, n: (G,) node counts (device int32 or host ints).

    Returns a ``GraphBatch`` with ``src``/``dst`` (sum E,) int32 (node ids g*nmax + i),
    ``pseudo`` (sum E, 2) fp32, ``edge_off`` (G+1,) int64 (device) and ``edge_off_host``,
    ``ecount`` (G,) int32, ``deg`` (G, nmax) int32, ``adj`` bit rows, optional dense ``A``
    (G, nmax, nmax) fp32 and incidence ``Ginc``/``Hinc`` (G, nmax, epad) fp32.
    The only host synchronisation is the read-back of the G edge counts (to size the edge list)."""
    if stg not in STRATEGIES:
        raise ValueError("No strategy named {} found.".format(stg))
    _dev(P)
    if P.dim() != 3 or P.shape[-1] != 2 or P.dtype != torch.float32:
        raise _lib.FpmError("build_graph_batch: P must be (G, nmax, 2) float32")
    P = P.contiguous()
    Gn, nmax = int(P.shape[0]), int(P.shape[1])
    dev = P.device
    n = torch.as_tensor(n, dtype=torch.int32).to(dev).contiguous()
    if n.numel() != Gn:
        raise _lib.FpmError("build_graph_batch: need one node count per graph")
    lib = _lib.load()
    W = lib.fpm_graph_words(nmax)
    adj = torch.empty(Gn, nmax, W, dtype=torch.int32, device=dev)
    deg = torch.empty(Gn, nmax, dtype=torch.int32, device=dev)
    ecount = torch.empty(Gn, dtype=torch.int32, device=dev)
    A = torch.empty(Gn, nmax, nmax, dtype=torch.float32, device=dev) if want_A else None
    st = _stream(P)
    _check(lib.fpm_graph_build(_p(P), _p(n), Gn, nmax, STRATEGIES[stg], float(thre), _p(adj), _p(deg), _p(ecount),
                               _p(A), st))
    ec_host = ecount.cpu()
    E = int(ec_host.sum())
    src = torch.empty(E, dtype=torch.int32, device=dev)
    dst = torch.empty(E, dtype=torch.int32, device=dev)
    pseudo = torch.empty(E, 2, dtype=torch.float32, device=dev)
    edge_off = torch.empty(Gn + 1, dtype=torch.int64, device=dev)
    Ginc = Hinc = None
    if want_GH:
        epad = int(ec_host.max()) if epad is None else int(epad)
        if Gn and epad < int(ec_host.max()):
            raise _lib.FpmError("build_graph_batch: edge_pad %d < edge_num %d" % (epad, int(ec_host.max())))
        Ginc = torch.zeros(Gn, nmax, epad, dtype=torch.float32, device=dev)
        Hinc = torch.zeros(Gn, nmax, epad, dtype=torch.float32, device=dev)
    _check(lib.fpm_graph_edges(_p(P), _p(adj), _p(deg), _p(ecount), Gn, nmax, float(rescale), _p(src), _p(dst),
                               _p(pseudo), _p(edge_off), _p(Ginc), _p(Hinc), int(epad or 0), st))
    off_host = torch.cat([torch.zeros(1, dtype=torch.int64), ec_host.to(torch.int64).cumsum(0)])
    return GraphBatch(src=src, dst=dst, pseudo=pseudo, edge_off=edge_off, edge_off_host=off_host, ecount=ecount,
                      deg=deg, adj=adj, A=A, Ginc=Ginc, Hinc=Hinc, nmax=nmax, n=n)


def build_graphs(P, n, n_pad=None, edge_pad=None, stg="fc", sym=True, thre=0):
    """``utils/build_graphs.py:12-74`` on the device: (A, G, H, edge_num) for one graph.

    P: (>= n, 2) keypoints (device tensor or array-like; computed on the current CUDA device)."""
    if not sym:
        raise NotImplementedError("build_graphs: only sym=True (the reference's SYM_ADJACENCY) is supported")
    P = torch.as_tensor(P)
    dev = P.device if P.is_cuda else torch.device("cuda")
    P = P[:n].to(device=dev, dtype=torch.float32).reshape(1, n, 2)
    gb = build_graph_batch(P, [n], stg=stg, thre=thre, want_A=True, want_GH=True, epad=edge_pad)
    edge_num = int(gb.edge_off_host[1])
    if edge_num <= 0 or n <= 0:
        raise AssertionError("Error in n = {} and edge_num = {}".format(n, edge_num))
    n_pad = n if n_pad is None else n_pad
    if n_pad < n:
        raise AssertionError("n_pad < n")
    A = gb.A[0]
    Gm, Hm = gb.Ginc[0], gb.Hinc[0]
    if n_pad > n:
        Gm = torch.nn.functional.pad(Gm, (0, 0, 0, n_pad - n))
        Hm = torch.nn.functional.pad(Hm, (0, 0, 0, n_pad - n))
    return A, Gm, Hm, edge_num


def kronecker_pattern(src1, dst1, src2, dst2, n1pad, base1=0, base2=0, dtype=torch.float32):
    """KGHs_sparse of one pair (gmdataset.py:623-634): (rowG, colH) over the E1*E2 edge pairs in
    kron(G2, G1) column order; node ids are shifted by -base1/-base2 (batch-global -> local).
    float32 like the reference's ``.float()`` use in ngm.py:339, or int64."""
    _dev(src1, dst1, src2, dst2)
    for t in (src1, dst1, src2, dst2):
        if t.dtype != torch.int32:
            raise _lib.FpmError("kronecker_pattern: edge ids must be int32")
    E1, E2 = int(src1.numel()), int(src2.numel())
    if dtype not in (torch.float32, torch.int64):
        raise _lib.FpmError("kronecker_pattern: dtype must be float32 or int64")
    rowG = torch.empty(E1 * E2, dtype=dtype, device=src1.device)
    colH = torch.empty(E1 * E2, dtype=dtype, device=src1.device)
    lib = _lib.load()
    _check(lib.fpm_kron_pattern(_p(src1.contiguous()), _p(dst1.contiguous()), E1, _p(src2.contiguous()),
                                _p(dst2.contiguous()), E2, int(base1), int(base2), int(n1pad),
                                0 if dtype == torch.float32 else 1, _p(rowG), _p(colH), _stream(src1)))
    return rowG, colH


__all__ = ["build_graph_batch", "build_graphs", "kronecker_pattern", "GraphBatch", "STRATEGIES"]
