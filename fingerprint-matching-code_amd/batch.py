"""Device-side batch layout for the matcher's forward.

Per side g (0 = source graphs ``idx1``, 1 = target graphs ``idx2``):
  * x[g]      (B*nmax_g, 768) fp32   node features, graph b at rows [b*nmax_g, b*nmax_g + n_b),
                                     zero rows in the padding (the reference concatenates unpadded
                                     graphs in a PyG Batch, ngm.py:246-251; padding is inert here);
  * src/dst[g] (E_g,) int32          edges with padded global node ids (PyG message flow src -> dst);
  * pseudo[g] (E_g, 2) fp32          edge_attr pseudo-coordinates (GMDataset.to_pyg_graph);
  * w[g]      (B, 512) fp32          global feature (ngm.py:238).
n1/n2 are per-pair node counts (int32, device + host copies); n1max/n2max the batch maxima.
"""
import os

import numpy as np
import torch

from . import config as C

# graph-2 block order of the GNN layers (a schedule; results unchanged): boxes over this many
# keypoints run their (pair, graph-2 node) workgroups in Hilbert-curve order of the keypoints, so the
# workgroups in flight share neighbour rows in L2 (n = 512: -15 % per 17-channel layer, no effect at
# n = 256 where a pair's state fits the L2 anyway; profiles/r06_gnn_order.txt)
ORDER_MIN_NMAX = 256
# FPM_GNN_ORDER=0: identity block order everywhere (A/B)
ORDER_ON = os.environ.get("FPM_GNN_ORDER", "1") != "0"


def hilbert_order(P, n, nmax):
    """(B, nmax) int32 permutation per pair: valid keypoints P[b, :n[b]] (x in [0, 320), y in
    [0, 240), the reference's frame) in Hilbert-curve order, then the padding slots in index order.
    Vectorised torch on P's device."""
    P = torch.as_tensor(P, dtype=torch.float32)
    B = P.shape[0]
    n = torch.as_tensor(n, dtype=torch.int64, device=P.device).view(B, 1)
    q = torch.stack([P[..., 0] / 320.0, P[..., 1] / 240.0], -1).clamp(0.0, 1.0) * 1023.0
    x, y = q[..., 0].long(), q[..., 1].long()
    d = torch.zeros_like(x)
    s = 512
    while s > 0:
        rx, ry = (x & s) > 0, (y & s) > 0
        d += s * s * ((3 * rx.long()) ^ ry.long())
        m = ~ry
        sw = m & rx
        x = torch.where(sw, 1023 - x, x)
        y = torch.where(sw, 1023 - y, y)
        x, y = torch.where(m, y, x), torch.where(m, x, y)
        s >>= 1
    idx = torch.arange(nmax, device=P.device).view(1, nmax).expand(B, nmax)
    key = torch.where(idx < n, d, (1 << 21) + idx)      # padding after every valid key, in index order
    return torch.argsort(key, dim=1, stable=True).to(torch.int32).contiguous()


class DeviceBatch:
    def __init__(self, B, n1, n2, x, w, src, dst, pseudo, device, nmax=None, edge_off=None, shared0=False):
        self.B = B
        # probe x gallery (C4): every pair's side-0 graph is the same probe; its per-graph stage
        # (SplineConv) is computed once per (sub-)batch and broadcast
        self.shared0 = shared0
        self.device = device
        self.n_host = [torch.as_tensor(n1, dtype=torch.int32), torch.as_tensor(n2, dtype=torch.int32)]
        self.n = [t.to(device) for t in self.n_host]
        # padded sizes; a sub-batch keeps its parent's (results depend on the batch maxima, quirk A.10(iii))
        self.nmax = list(nmax) if nmax is not None else [int(self.n_host[0].max()), int(self.n_host[1].max())]
        self.x, self.w, self.src, self.dst, self.pseudo = x, w, src, dst, pseudo
        self.E = [int(s.numel()) for s in src]
        # per side, cumulative edge offsets per pair (host), for splitting into sub-batches
        self.edge_off = edge_off
        self._splits = {}
        # optional (B, n2max) int32 graph-2 block order of the GNN layers (hilbert_order; None = identity)
        self.ord2 = None

    def split(self, k, tail=0):
        """k contiguous sub-batches of pairs (views of x/w, renumbered edge copies); cached.
        ``tail`` > 0 halves the last chunk ``tail`` times (a short final chunk shortens the host
        Hungarian that runs after the GPU has finished).  (Halving the last two chunks as equal
        pairs -- 64, 64, 32, 32, ... -- shortened that tail but slowed the GPU stage 2-4 % with the
        extra chunks: profiles/r03l_tail_split_ab.txt.)"""
        if k <= 1 or self.B < 2:
            return [self]
        key = (k, tail)
        if key in self._splits:
            return self._splits[key]
        if self.edge_off is None:
            raise ValueError("split() needs per-pair edge offsets")
        bounds = [round(i * self.B / k) for i in range(k + 1)]
        for _ in range(tail):
            a, b = bounds[-2], bounds[-1]
            if b - a >= 2:
                bounds.insert(-1, (a + b) // 2)
        parts = [self.split_range(bounds[c], bounds[c + 1]) for c in range(len(bounds) - 1)
                 if bounds[c + 1] > bounds[c]]
        self._splits[key] = parts
        return parts

    def split_range(self, b0, b1):
        """Pairs [b0, b1) as a sub-batch (views of x/w, renumbered edge copies) that keeps this
        batch's padded sizes; ``pair_range`` records where it sits in the parent."""
        if self.edge_off is None:
            raise ValueError("split_range() needs per-pair edge offsets")
        if not 0 <= b0 < b1 <= self.B:
            raise ValueError("split_range: bad pair range [%d, %d) of %d" % (b0, b1, self.B))
        xs, ws, ss, ds, ps = [], [], [], [], []
        for side in range(2):
            nm = self.nmax[side]
            e0, e1 = int(self.edge_off[side][b0]), int(self.edge_off[side][b1])
            xs.append(self.x[side][b0 * nm:b1 * nm])
            ws.append(self.w[side][b0:b1])
            ss.append((self.src[side][e0:e1] - b0 * nm).contiguous())
            ds.append((self.dst[side][e0:e1] - b0 * nm).contiguous())
            ps.append(self.pseudo[side][e0:e1])
        eo = [self.edge_off[side][b0:b1 + 1] - self.edge_off[side][b0] for side in range(2)]
        sub = DeviceBatch(b1 - b0, self.n_host[0][b0:b1], self.n_host[1][b0:b1], xs, ws, ss, ds, ps, self.device,
                          nmax=self.nmax, edge_off=eo, shared0=self.shared0)
        sub.pair_range = (b0, b1)
        sub.ord2 = None if self.ord2 is None else self.ord2[b0:b1]
        return sub

    def to(self, device, non_blocking=True):
        """The same batch on another device (peer copies of features, edges and counts); keeps the
        padded sizes, so a shard computed there equals its slice of the parent batch bit for bit."""
        device = torch.device(device)
        if device == self.device:
            return self
        mv = lambda ts: [t.to(device, non_blocking=non_blocking) for t in ts]
        out = DeviceBatch(self.B, self.n_host[0], self.n_host[1], mv(self.x), mv(self.w), mv(self.src), mv(self.dst),
                          mv(self.pseudo), device, nmax=self.nmax, edge_off=self.edge_off, shared0=self.shared0)
        if hasattr(self, "pair_range"):
            out.pair_range = self.pair_range
        out.ord2 = None if self.ord2 is None else self.ord2.to(device, non_blocking=non_blocking)
        return out

    def max_graph_edges(self, side):
        """Largest edge count of one graph on ``side`` (host edge offsets; 0 when unknown): lets the
        spline plan use its per-graph kernels."""
        if self.edge_off is None:
            return 0
        off = torch.as_tensor(self.edge_off[side])
        return int((off[1:] - off[:-1]).max()) if off.numel() > 1 else 0

    @property
    def n1(self):
        return self.n[0]

    @property
    def n2(self):
        return self.n[1]

    @property
    def n1max(self):
        return self.nmax[0]

    @property
    def n2max(self):
        return self.nmax[1]

    @staticmethod
    def from_pairs(pairs, device):
        """From ``fpm.synth`` pairs (list of (g0, g1) dicts)."""
        B = len(pairs)
        xs, ws, srcs, dsts, pss = [], [], [], [], []
        ns, eoffs = [], []
        for side in range(2):
            n = np.array([p[side]["n"] for p in pairs], dtype=np.int32)
            eoffs.append(torch.from_numpy(np.concatenate(
                [[0], np.cumsum([p[side]["edge_index"].shape[1] for p in pairs])]).astype(np.int64)))
            nmax = int(n.max())
            X = np.zeros((B, nmax, C.NODE_FEATURE_DIM), np.float32)
            s_l, d_l, p_l = [], [], []
            for b, p in enumerate(pairs):
                g = p[side]
                X[b, :g["n"]] = g["x"]
                ei = g["edge_index"]
                s_l.append(ei[0] + b * nmax)
                d_l.append(ei[1] + b * nmax)
                p_l.append(g["pseudo"])
            ns.append(n)
            xs.append(torch.from_numpy(X.reshape(B * nmax, -1)).to(device))
            ws.append(torch.from_numpy(np.stack([p[side]["w"] for p in pairs]).astype(np.float32)).to(device))
            srcs.append(torch.from_numpy(np.concatenate(s_l).astype(np.int32)).to(device))
            dsts.append(torch.from_numpy(np.concatenate(d_l).astype(np.int32)).to(device))
            pss.append(torch.from_numpy(np.concatenate(p_l).astype(np.float32)).to(device).contiguous())
        bt = DeviceBatch(B, ns[0], ns[1], xs, ws, srcs, dsts, pss, device, edge_off=eoffs)
        if ORDER_ON and bt.nmax[1] > ORDER_MIN_NMAX and all("P" in p[1] for p in pairs):
            P2 = np.zeros((B, bt.nmax[1], 2), np.float32)
            for b, p in enumerate(pairs):
                P2[b, :p[1]["n"]] = p[1]["P"]
            bt.ord2 = hilbert_order(torch.from_numpy(P2), ns[1], bt.nmax[1]).to(device)
        return bt

    @staticmethod
    def from_keypoints(P, n, x, w, device, stg="tri"):
        """Keypoints straight to a device batch: both sides' graphs are built on the GPU
        (``fpm.graphs``: Delaunay adjacency, np.nonzero edge order, pseudo-coordinates), as the
        reference's DataLoader does on the host (gmdataset.py:233-244, build_graphs.py:77-100).

        P: 2 x (B, nmax_g, 2) fp32 keypoints; n: 2 x (B,) node counts; x: 2 x (B*nmax_g, 768) fp32
        node features (zero padding rows); w: 2 x (B, 512) global features."""
        from . import graphs
        B = int(P[0].shape[0])
        srcs, dsts, pss, eoffs, ns = [], [], [], [], []
        for side in range(2):
            gb = graphs.build_graph_batch(P[side].to(device), n[side], stg=stg)
            srcs.append(gb.src)
            dsts.append(gb.dst)
            pss.append(gb.pseudo)
            eoffs.append(gb.edge_off_host)
            ns.append(torch.as_tensor(n[side], dtype=torch.int32).cpu())
        bt = DeviceBatch(B, ns[0], ns[1], [x[0], x[1]], [w[0], w[1]], srcs, dsts, pss, device,
                         nmax=[int(P[0].shape[1]), int(P[1].shape[1])], edge_off=eoffs)
        if ORDER_ON and bt.nmax[1] > ORDER_MIN_NMAX:
            bt.ord2 = hilbert_order(P[1].to(device), ns[1], bt.nmax[1])
        return bt

    @staticmethod
    def from_probe_gallery(probe, gallery, device):
        """One probe graph against a gallery (C4): pairs (probe, g) with the probe's
        per-graph stage shared.  Inputs are staged per pair (simple layout); compute is not."""
        bt = DeviceBatch.from_pairs([(probe, g) for g in gallery], device)
        bt.shared0 = True
        return bt

    @staticmethod
    def from_data_dict(data_dict, device):
        """From a reference-shaped data_dict with the synthetic bypass keys.

        Reads ``ns`` (2 x (B,)), ``pyg_graphs`` (2 duck-typed PyG batches: edge_index (2, sumE) with
        unpadded batch-global node ids, edge_attr (sumE, 2), and ``ptr`` or ``batch``),
        ``node_features`` (2 x (B, nmax, 768) padded or (sum n, 768) concatenated) and
        ``global_features`` (2 x (B, 512)).  Backbone features from ``images`` are out of scope.
        """
        if "node_features" not in data_dict:
            raise NotImplementedError(
                "fpm.Net starts after the ResNet-18 backbone + feature_align (out of scope, see DESIGN.md): "
                "pass data_dict['node_features'] and data_dict['global_features']")
        ns = [torch.as_tensor(t).view(-1).to(torch.int32).cpu() for t in data_dict["ns"]]
        B = int(ns[0].numel())
        xs, ws, srcs, dsts, pss, eoffs = [], [], [], [], [], []
        for side in range(2):
            n = ns[side]
            nmax = int(n.max())
            g = data_dict["pyg_graphs"][side]
            ptr = getattr(g, "ptr", None)
            if ptr is None:
                counts = torch.bincount(torch.as_tensor(g.batch).cpu(), minlength=B)
                ptr = torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)])
            ptr = torch.as_tensor(ptr).cpu().long()
            ei = torch.as_tensor(g.edge_index).cpu().long()
            gidx = torch.searchsorted(ptr, ei[0], right=True) - 1
            if ei.shape[1] and not bool((gidx[1:] >= gidx[:-1]).all()):
                order = torch.argsort(gidx, stable=True)
                ei, gidx = ei[:, order], gidx[order]
                g_attr = torch.as_tensor(g.edge_attr)[order]
            else:
                g_attr = torch.as_tensor(g.edge_attr)
            eoffs.append(torch.cat([torch.zeros(1, dtype=torch.long), torch.bincount(gidx, minlength=B).cumsum(0)]))
            off = gidx * nmax - ptr[gidx]
            srcs.append((ei[0] + off).to(torch.int32).to(device))
            dsts.append((ei[1] + off).to(torch.int32).to(device))
            pss.append(g_attr.to(torch.float32).to(device).contiguous())
            nf = torch.as_tensor(data_dict["node_features"][side]).to(torch.float32)
            if nf.dim() == 3:
                X = torch.zeros(B, nmax, nf.shape[-1], dtype=torch.float32, device=nf.device)
                X[:, :nf.shape[1]] = nf[:, :nmax]
                keep = torch.arange(nmax, device=nf.device)[None, :] < n.to(nf.device).view(-1, 1)
                X = torch.where(keep[..., None], X, torch.zeros((), device=nf.device))
            else:
                X = torch.zeros(B, nmax, nf.shape[-1], dtype=torch.float32, device=nf.device)
                for b in range(B):
                    X[b, :int(n[b])] = nf[int(ptr[b]):int(ptr[b + 1])]
            xs.append(X.reshape(B * nmax, -1).to(device).contiguous())
            ws.append(torch.as_tensor(data_dict["global_features"][side]).to(torch.float32).to(device).contiguous())
        return DeviceBatch(B, ns[0], ns[1], xs, ws, srcs, dsts, pss, device, edge_off=eoffs)
