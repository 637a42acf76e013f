"""``Net``: the fingerprint QAP matcher's graph-matching forward on MI355X.

Drop-in for the reference's ``Net`` (``src/model/ngm.py:117-491``): same constructor
(``Net(regression=False)``), same ``forward(data_dict, regression=True) -> data_dict`` writing
``ds_mat``, ``perm_mat``, ``ks_loss``, ``ks_error``, ``cls_loss``, ``cls_prob``, ``k_prob``
(ngm.py:479-487), and the same state_dict names/shapes (so ``utils/models_sl.load_model`` works).
Like the reference's ``Net`` (ngm.py:226-249), the default constructor carries the ResNet-18
backbone (``node_layers.*`` / ``edge_layers.*`` state_dict names), so the reference's
``images`` / ``Ps`` / ``ns`` data_dict (``evaluate_binary_classifier.py:77-97``) works as is:
ResNet-18 on MIOpen (``fpm.backbone``), then the fused normalise + feature_align + concat kernel
(``fpm_feature_align_fwd``); missing ``pyg_graphs`` are built on the device from ``Ps``
(Delaunay, ``fpm.graphs``).  A data_dict that already holds per-graph node features
(``node_features`` / ``global_features``, or a prebuilt ``fpm_batch``) skips the backbone;
``Net(backbone=False)`` builds the matcher alone (its state_dict then has no backbone keys).
Every compute stage runs in ``libfpm_hip.so``; the
Hungarian step runs on host threads (``fpm_lsa_batch_host``) as the reference's does.

``dtype``: ``"f32"`` (parity mode: fp32 MFMA, matches the CPU oracle) or ``"bf16"`` (bf16 MFMA
operands with fp32 accumulation for the GEMMs; everything else fp32).
"""
import os
import time

import numpy as np

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import config as C
from . import ops
from . import params as P
from .batch import DeviceBatch


def host_cpu_share():
    """CPUs this process may use for the host Hungarian pool.  ``FPM_CPU_SHARE`` sets it explicitly
    (``FPM_LSA_THREADS`` sets the pool size itself, default 2 per CPU of the share).  Otherwise:
    OMP_NUM_THREADS (16 per GPU on the pool) capped by the affinity mask; under
    torch.distributed.run (LOCAL_WORLD_SIZE present), whose launcher exports OMP_NUM_THREADS=1 when
    the variable was unset, a share of 1 is read as that default and replaced by the affinity mask
    split over the node's ranks (at most 16 each) -- set FPM_CPU_SHARE=1 to really run on one CPU."""
    n_aff = len(os.sched_getaffinity(0))
    if os.environ.get("FPM_CPU_SHARE"):
        return max(1, min(int(os.environ["FPM_CPU_SHARE"]), n_aff))
    omp = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    if omp <= 1 and "LOCAL_WORLD_SIZE" in os.environ:
        omp = min(16, n_aff // max(1, int(os.environ["LOCAL_WORLD_SIZE"])))
    return max(1, min(omp, n_aff))


class _Node(nn.Module):
    pass


def _build_tree(root, sd):
    """Register every state_dict entry under its dotted name (float tensors as Parameters)."""
    for name, t in sd.items():
        parts = name.split(".")
        m = root
        for p in parts[:-1]:
            if not hasattr(m, p) or not isinstance(getattr(m, p), nn.Module):
                m.add_module(p, _Node())
            m = getattr(m, p)
        leaf = parts[-1]
        is_buf = (not t.is_floating_point()) or leaf in ("running_mean", "running_var")
        if is_buf:
            m.register_buffer(leaf, t.clone())
        else:
            m.register_parameter(leaf, nn.Parameter(t.clone()))


class Net(nn.Module):
    def __init__(self, regression=False, dtype="f32", seed=0, lsa_threads=None, chunks=None, compute_ke=False,
                 backbone=True, lsa=None):
        super().__init__()
        _build_tree(self, P.init_params(seed))
        if backbone:
            # ResNet18_final split (feature_extractor.py:7-75), reference parameter names
            from .backbone import build_resnet18_split
            self.node_layers, self.edge_layers, self.final_layers = build_resnet18_split(seed)
        # train.py's parameter groups (train.py:157-239).  backbone_params: the backbone's own
        # parameters (feature_extractor.py:19 takes list(self.parameters()) before the matcher
        # modules exist); k_params_id / k_params: encoder_k + final_row + final_col (ngm.py:174-199)
        self.backbone_params = ([p for m in (self.node_layers, self.edge_layers, self.final_layers)
                                 for p in m.parameters()] if backbone else [])
        self.k_params_id = [id(p) for m in self._k_modules() for p in m.parameters()]
        self._backbone_dev = None
        # Hungarian step (utils/hungarian.py): "host" = C++ thread pool over a pinned ds_mat copy,
        # "device" = the same solver restated per wavefront (fpm_lsa_batch_device, bit-identical)
        self.lsa_mode = lsa or os.environ.get("FPM_LSA", "host")
        if self.lsa_mode not in ("host", "device"):
            raise ValueError("lsa must be 'host' or 'device'")
        self.regression = regression
        self.mean_k = True
        self.tau = C.SK_TAU
        self.univ_size = C.UNIV_SIZE
        self.k_factor = C.K_FACTOR
        if dtype not in ("f32", "bf16"):
            raise ValueError("dtype must be 'f32' or 'bf16'")
        self.dtype_mode = dtype
        # AFA-U operands in the bf16 mode (FPM_AFAU_DTYPE): "bf16s" (default) keeps the attention
        # output as split bf16 hi + lo terms for the multi-head combine product and runs the FFN on
        # bf16; "bf16" rounds the attention output to bf16 (k_prob 8e-3 from the fp32 oracle at C3
        # vs 8e-4, perm_mat tie-equivalent on 1-2 of 8 vs 7 of 8 pairs, 1 % faster); "bf16x3" /
        # "f32" every AFA-U product near-fp32 / fp32 (15-19 % slower end to end).
        self.afau_mode = "f32" if dtype == "f32" else os.environ.get("FPM_AFAU_DTYPE", "bf16s")
        if self.afau_mode not in ("f32", "bf16", "bf16s", "bf16x3"):
            raise ValueError("FPM_AFAU_DTYPE must be f32, bf16, bf16s or bf16x3")
        # Hungarian pool: 2 threads per CPU of the process's share (FPM_LSA_THREADS overrides).  Measured
        # on the 16-CPU box share: 16 / 32 / 48 threads -> 29-44 / 17-22 / 17-18 ms per 1024 pairs
        # (the pairs of a chunk differ in cost; idle stragglers at each chunk's join dominate at 1x)
        share = host_cpu_share()
        self.lsa_threads = lsa_threads or int(os.environ.get("FPM_LSA_THREADS", str(2 * share)))
        self.chunks = chunks
        # quadratic (edge) affinity Ke (ngm.py:282-289): dead for every output, off by default
        self.compute_ke = compute_ke
        self._pack = None
        self._pack_key = None
        self._pinned = None
        self._stream_cache = {}
        self.n_streams = max(1, int(os.environ.get("FPM_STREAMS", "2")))
        self.tail_splits = int(os.environ.get("FPM_TAIL", "2"))
        self.head_splits = int(os.environ.get("FPM_HEAD", "0"))
        # FPM_ZERO_COPY=1: soft_topk writes ds_mat straight into pinned host memory instead of a
        # stream copy.  Measured slower (21.2K -> 19.7K pairs/s: the kernel stalls on PCIe writes
        # on the critical path), so off by default.
        self.zero_copy = os.environ.get("FPM_ZERO_COPY", "0") == "1"
        self.copy_stream = os.environ.get("FPM_COPY_STREAM", "1") == "1"
        # > 0: ds_mat D2H on this many workgroups (fpm_copy_async) instead of the runtime's blit
        self.copy_blocks = int(os.environ.get("FPM_COPY_BLOCKS", "0"))
        # > 0: ds_mat D2H through hipMemcpyAsync with this copy kind (fpm_memcpy_async; 1024 = the
        # no-compute-unit device-to-device kind, i.e. a copy engine instead of the blit kernel)
        self.copy_kind = int(os.environ.get("FPM_COPY_KIND", "0"))
        # defer each chunk's ds_mat D2H until the side-0 spline plan of the chunk queued two places
        # later (same compute stream) has run: that latency-bound kernel otherwise runs beside the
        # copy's blit kernel and stalls ~25x
        self.copy_defer = int(os.environ.get("FPM_COPY_DEFER", "1"))
        if self.copy_defer not in (0, 1):
            raise ValueError("FPM_COPY_DEFER must be 0 or 1")
        self._plan_events = None
        # FPM_OFFSET=1: the second stream starts its first chunk after the first chunk's SplineConv,
        # so the streams' phases interleave (MFMA-heavy SplineConv beside the VALU / memory-bound GNN,
        # Sinkhorn and soft top-k) instead of running the same stages side by side
        self.stream_offset = int(os.environ.get("FPM_OFFSET", "0"))
        self._offset_events = None
        # the host thread waits for each chunk's ds_mat with a sleeping (not spinning) event wait,
        # leaving its core to the Hungarian pool
        self.blocking_wait = os.environ.get("FPM_BLOCKING_WAIT", "1") == "1"
        self._keep_feats = False
        self._stage_timing = os.environ.get("FPM_STAGE_TIMING", "0") == "1"
        self.stage_times = {}
        self._t_last = 0.0
        self.last_timing = {}
        self.eval()

    # ------------------------------------------------------------------------------------------
    def _k_modules(self):
        return (self.encoder_k, self.final_row, self.final_col)

    @property
    def k_params(self):
        """The k regressor's optimizer groups (ngm.py:195-199): encoder_k, final_row, final_col.
        The reference stores generators (consumed by the first pass over them); every access here
        returns fresh lists of the same parameters, so stage 1's freeze loop and a later
        ``optim.AdamW(model.k_params)`` both see them."""
        return [{"params": list(m.parameters())} for m in self._k_modules()]

    def _sd(self):
        return dict(self.state_dict())

    def _key(self, device):
        return (str(device), self.dtype_mode, self.afau_mode, tuple(p._version for p in self.parameters()),
                tuple(b._version for b in self.buffers()))

    def packed(self, device):
        """Device-resident, kernel-layout copies of the parameters (rebuilt if they change)."""
        key = self._key(device)
        if self._pack is not None and self._pack_key == key:
            return self._pack
        sd = {k: v.detach() for k, v in self.state_dict().items()}
        op = torch.bfloat16 if self.dtype_mode == "bf16" else torch.float32
        d = {}
        g = lambda k: sd[k].to(device=device, dtype=torch.float32).contiguous()
        for l in range(2):
            pre = "%s.%d" % (P.SPLINE_PREFIX, l)
            # [cell][out][in] for the 25 spline cells, then the root weight as cell 25
            d["W%d" % l] = torch.cat([sd[pre + ".weight"].to(device).transpose(1, 2),
                                      sd[pre + ".root"].to(device).t()[None]]).contiguous().to(op)
            d["bias%d" % l] = g(pre + ".bias")
        d["aff_w"] = g("vertex_affinity.A.weight")          # [768][1024] = N x K
        d["aff_b"] = g("vertex_affinity.A.bias")
        d["eaff_w"] = g("edge_affinity.A.weight")
        d["eaff_b"] = g("edge_affinity.A.bias")
        for l in range(C.GNN_LAYER):
            pre = "gnn_layer_%d" % l
            # kernel layout (gnn.hip GnnPack): weight matrices transposed to [in][out]
            parts = [sd[pre + ".conv2.lin_l.weight"].t(), sd[pre + ".conv2.lin_l.bias"], sd[pre + ".conv2.lin_r.weight"].t(),
                     sd[pre + ".n_self_func.0.weight"].t(), sd[pre + ".n_self_func.0.bias"],
                     sd[pre + ".n_self_func.2.weight"].t(), sd[pre + ".n_self_func.2.bias"],
                     sd[pre + ".classifier.weight"], sd[pre + ".classifier.bias"]]
            d["gnn%d" % l] = torch.cat([t.reshape(-1).float() for t in parts]).to(device).contiguous()
        d["cls_w"] = g("classifier.weight").reshape(-1).contiguous()
        d["cls_b"] = g("classifier.bias")
        op = torch.bfloat16 if self.afau_mode == "bf16" else torch.float32
        for blk in ("row", "col"):
            pre = "encoder_k.layers.0.%s_encoding_block" % blk
            d[blk + "_Wv"] = g(pre + ".Wv.weight")                                  # (256, 600)
            d[blk + "_mix1w"] = g(pre + ".mixed_score_MHA.mix1_weight")
            d[blk + "_mix1b"] = g(pre + ".mixed_score_MHA.mix1_bias")
            d[blk + "_mix2w"] = g(pre + ".mixed_score_MHA.mix2_weight")
            d[blk + "_mix2b"] = g(pre + ".mixed_score_MHA.mix2_bias")
            Wc = sd[pre + ".multi_head_combine.weight"].to(device)                                   # (600, 256)
            W1 = sd[pre + ".feed_forward.W1.weight"].to(device)                                      # (256, 600)
            W2 = sd[pre + ".feed_forward.W2.weight"].to(device)                                      # (600, 256)
            if self.afau_mode == "bf16s":
                # the combine product on split operands ([W_hi | W_hi | W_lo]); FFN plain bf16
                d[blk + "_Wc"] = ops.split_weights_bf16x3(Wc, C.AFAU_HEADS * C.AFAU_QKV)
                d[blk + "_W1"] = F.pad(W1, (0, C.AFAU_EMB_PAD - C.AFAU_EMB)).contiguous().to(torch.bfloat16)
                d[blk + "_W2"] = W2.contiguous().to(torch.bfloat16)
            elif self.afau_mode == "bf16x3":
                # [W_hi | W_hi | W_lo] along K for the split-bf16 operands (ops.split_bf16x3)
                d[blk + "_Wc"] = ops.split_weights_bf16x3(Wc, C.AFAU_HEADS * C.AFAU_QKV)
                d[blk + "_W1"] = ops.split_weights_bf16x3(W1, C.AFAU_EMB_PAD)
                d[blk + "_W2"] = ops.split_weights_bf16x3(W2, C.AFAU_FF)
            else:
                if op == torch.bfloat16:      # K padded with zeros to the 256-row kernel's BK multiple
                    W1 = F.pad(W1, (0, C.AFAU_EMB_PAD - C.AFAU_EMB))
                d[blk + "_Wc"] = Wc.contiguous().to(op)
                d[blk + "_W1"] = W1.contiguous().to(op)
                d[blk + "_W2"] = W2.contiguous().to(op)
            d[blk + "_bc"] = g(pre + ".multi_head_combine.bias")
            d[blk + "_b1"] = g(pre + ".feed_forward.W1.bias")
            d[blk + "_b2"] = g(pre + ".feed_forward.W2.bias")
            for k in (1, 2):
                d["%s_n%dw" % (blk, k)] = g(pre + ".add_n_normalization_%d.norm.weight" % k)
                d["%s_n%db" % (blk, k)] = g(pre + ".add_n_normalization_%d.norm.bias" % k)
        for h in ("final_row", "final_col"):
            for i in (0, 2):
                d["%s%dw" % (h, i)] = g("%s.%d.weight" % (h, i)).reshape(-1).contiguous()
                d["%s%db" % (h, i)] = g("%s.%d.bias" % (h, i))
        for ci, bi, tag in ((0, 2, "1"), (4, 6, "2")):
            d["mc_w" + tag] = g("match_cls.conv.%d.weight" % ci).reshape(-1).contiguous()
            d["mc_b" + tag] = g("match_cls.conv.%d.bias" % ci)
            rm, rv = sd["match_cls.conv.%d.running_mean" % bi].double(), sd["match_cls.conv.%d.running_var" % bi].double()
            gw, gb = sd["match_cls.conv.%d.weight" % bi].double(), sd["match_cls.conv.%d.bias" % bi].double()
            sc = gw / torch.sqrt(rv + C.BN_EPS)
            d["mc_sc" + tag] = sc.float().to(device)
            d["mc_sh" + tag] = (gb - rm * sc).float().to(device)
        d["mc_fcw"] = g("match_cls.fc.weight").reshape(-1).contiguous()
        d["mc_fcb"] = g("match_cls.fc.bias")
        self._pack, self._pack_key = d, key
        return d

    # ------------------------------------------------------------------------------------------
    def _spline_side(self, wp, bt, side, cscale, x_op=None):
        """SiameseSConvOnNodes over one side's batch (spline_conv.py:28-57) -> operand rows.
        ``x_op``: this side's bf16 operand rows when the caller cast the whole batch up front."""
        dev = bt.device
        op = torch.bfloat16 if self.dtype_mode == "bf16" else torch.float32
        nn_ = bt.B * bt.nmax[side]
        E = bt.E[side]
        plan = ops.spline_plan(bt.src[side], bt.dst[side], bt.pseudo[side], nn_, bt.nmax[side],
                               bt.max_graph_edges(side))
        # copy deferral: the previous-but-one chunk's D2H starts after this side-0 plan
        if side == 0 and self._plan_events is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self._plan_events.append(ev)
        if side == 0 and bt.shared0 and bt.B > 1:
            return (plan,) + self._spline_shared(wp, bt, cscale)
        x0 = bt.x[side]
        if x_op is None:
            x_op = ops.cast_bf16(x0) if op == torch.bfloat16 else x0
        yws = ops.spline_y_ws(ops.BF16 if op == torch.bfloat16 else ops.F32, E, nn_, dev)
        h = torch.empty(nn_, C.NODE_FEATURE_DIM, device=dev, dtype=op)
        ops.spline_conv(x_op, plan, E, nn_, bt.nmax[side], bt.n[side], wp["W0"], wp["bias0"], yws, 0, out_t=h)
        out = torch.empty(nn_, C.NODE_FEATURE_DIM, device=dev, dtype=op)
        outf = torch.empty(nn_, C.NODE_FEATURE_DIM, device=dev, dtype=torch.float32) if self._keep_feats else None
        ops.spline_conv(h, plan, E, nn_, bt.nmax[side], bt.n[side], wp["W1"], wp["bias1"], yws, 1, xres=x0,
                        cscale=cscale, out_f=outf, out_t=out)
        return plan, out, outf

    def _spline_shared(self, wp, bt, cscale):
        """Probe x gallery: the shared side-0 graph's two SplineConv layers once (pair 0's slice),
        then broadcast to all pairs with the per-pair coefficient scaling (fpm_rows_bcast_scale)."""
        dev = bt.device
        op = torch.bfloat16 if self.dtype_mode == "bf16" else torch.float32
        nm = bt.nmax[0]
        e0 = int(bt.edge_off[0][1])
        src, dst, ps = bt.src[0][:e0], bt.dst[0][:e0], bt.pseudo[0][:e0]
        plan = ops.spline_plan(src, dst, ps, nm, nm, e0)
        x0 = bt.x[0][:nm]
        nv = bt.n[0][:1]
        x_op = ops.cast_bf16(x0) if op == torch.bfloat16 else x0
        yws = ops.spline_y_ws(ops.BF16 if op == torch.bfloat16 else ops.F32, e0, nm, dev)
        h = torch.empty(nm, C.NODE_FEATURE_DIM, device=dev, dtype=op)
        ops.spline_conv(x_op, plan, e0, nm, nm, nv, wp["W0"], wp["bias0"], yws, 0, out_t=h)
        y = torch.empty(nm, C.NODE_FEATURE_DIM, device=dev, dtype=torch.float32)
        ops.spline_conv(h, plan, e0, nm, nm, nv, wp["W1"], wp["bias1"], yws, 1, xres=x0, out_f=y)
        out = torch.empty(bt.B * nm, C.NODE_FEATURE_DIM, device=dev, dtype=op)
        outf = torch.empty(bt.B * nm, C.NODE_FEATURE_DIM, device=dev, dtype=torch.float32) if self._keep_feats else None
        ops.rows_bcast_scale(y, bt.B, coef=cscale, out_f=outf, out_t=out)
        return out, outf

    def _afau_block(self, wp, blk, nb_, P_, mh=None, n2u_d=None):
        """One AFA-U encoder block's instance norms + FFN (afau.py:145-199) -> max over positions
        (nb_, E).  "row": on the attention-combine output mh; "col": the synthesised one-hot input
        C0 + combine bias of each distinct n2 (n2u_d)."""
        dev = wp["row_Wc"].device
        op = torch.bfloat16 if self.afau_mode in ("bf16", "bf16s") else torch.float32
        E, FF = C.AFAU_EMB, C.AFAU_FF
        x3 = self.afau_mode == "bf16x3"
        mask = int(os.environ.get("FPM_AFAU_X3_MASK", "7"))
        kx = lambda bit, kp: 3 * kp if mask & bit else kp
        rows = nb_ * P_
        o1f = torch.empty(rows, E, device=dev, dtype=torch.float32)
        KE = E if op == torch.float32 else C.AFAU_EMB_PAD      # bf16 operand copy: zero-padded K
        o1t = o1f if op == torch.float32 else torch.empty(rows, KE, device=dev, dtype=op)
        if blk == "row":
            ops.instnorm(mh, nb_, P_, E, wp["row_n1w"], wp["row_n1b"], out_f=o1f,
                         out_t=None if op == torch.float32 else o1t, ldt=KE)
        else:
            ops.instnorm(None, nb_, P_, E, wp["col_n1w"], wp["col_n1b"], nvalid=n2u_d, onehot_bias=wp["col_bc"],
                         out_f=o1f, out_t=None if op == torch.float32 else o1t, ldt=KE)
        ff = torch.empty(rows, E, device=dev, dtype=torch.float32)
        if x3:
            o13 = ops.split_bf16x3(o1f, C.AFAU_EMB_PAD)
            hf = torch.empty(rows, FF, device=dev, dtype=torch.float32)
            ops.gemm(o13, wp[blk + "_W1"], rows, FF, kx(2, C.AFAU_EMB_PAD), o13.shape[1], o13.shape[1],
                     epi=ops.EPI_RELU, bias=wp[blk + "_b1"], out_f=hf, ldc=FF)
            h3 = ops.split_bf16x3(hf, FF)
            ops.gemm(h3, wp[blk + "_W2"], rows, E, kx(4, FF), h3.shape[1], h3.shape[1], bias=wp[blk + "_b2"],
                     out_f=ff, ldc=E)
        else:
            hbuf = torch.empty(rows, FF, device=dev, dtype=op)
            ops.gemm(o1t, wp[blk + "_W1"], rows, FF, KE, KE, KE, epi=ops.EPI_RELU, bias=wp[blk + "_b1"],
                     out_t=hbuf if op != torch.float32 else None, out_f=hbuf if op == torch.float32 else None,
                     ldc=FF)
            ops.gemm(hbuf, wp[blk + "_W2"], rows, E, FF, FF, FF, bias=wp[blk + "_b2"], out_f=ff, ldc=E)
        gm = torch.empty(nb_, E, device=dev, dtype=torch.float32)
        ops.instnorm(o1f, nb_, P_, E, wp[blk + "_n2w"], wp[blk + "_n2b"], in2=ff, gmax=gm)
        return gm

    def _afau_col(self, wp, bt):
        """The AFA-U column block for every distinct n2 of a batch: (n2u, gmax per n2u, n2max).
        The column block sees a = one-hot rows and b = zero rows, so k = v = 0 and its attention
        output is exactly the combine bias (afau.py:99-142): its result depends on n2 and the batch's
        n2max only, not on ss.  A forward computes it once per distinct n2 and gathers it for every
        pair and pipeline chunk -- the same arithmetic on the same inputs, bit-identical to the
        per-pair evaluation."""
        if os.environ.get("FPM_AFAU_COLDEDUP", "1") == "1":
            n2u = np.unique(bt.n_host[1].numpy())
        else:
            n2u = bt.n_host[1].numpy()
        n2u_d = torch.as_tensor(n2u, dtype=torch.int32).to(bt.device, non_blocking=True)
        return n2u, self._afau_block(wp, "col", len(n2u), bt.n2max, n2u_d=n2u_d), bt.n2max

    def _afau(self, wp, ss, bt, col=None):
        """AFA-U k regression (ngm.py:386-412) -> ks (B,).  ``col``: the forward's _afau_col result
        (computed here for this batch when None)."""
        dev = ss.device
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        # f32 / bf16x3: fp32 activations; bf16 / bf16s: bf16 FFN operands
        op = torch.bfloat16 if self.afau_mode in ("bf16", "bf16s") else torch.float32
        E, HD = C.AFAU_EMB, C.AFAU_HEADS * C.AFAU_QKV
        if max(n1max, n2max) > self.univ_size:
            raise AssertionError("UNIV_SIZE cap: n1max/n2max must be <= %d (ngm.py:387-389)" % self.univ_size)
        x3 = self.afau_mode == "bf16x3"          # near-fp32 products on bf16 MFMA (split operands)
        split = self.afau_mode == "bf16s"        # the combine product alone on split operands
        att = torch.empty(B * n1max, 3 * HD if split else HD, device=dev,
                          dtype=torch.bfloat16 if split else op)
        ops.crossset_attn(ss, bt.n2, wp["row_Wv"], wp["row_mix1w"], wp["row_mix1b"], wp["row_mix2w"],
                          wp["row_mix2b"], att, split=split)
        mh = torch.empty(B * n1max, E, device=dev, dtype=torch.float32)
        # diagnostic: FPM_AFAU_X3_MASK selects which of (combine, W1, W2) use the three split terms;
        # the others multiply the hi parts only (plain bf16 products)
        mask = int(os.environ.get("FPM_AFAU_X3_MASK", "7"))
        kx = lambda bit, kp: 3 * kp if mask & bit else kp
        if x3:
            att = ops.split_bf16x3(att, HD)
        # bf16s: hi*W_hi + lo*W_hi (2 terms; the W_lo term changed nothing measurable, +0.7 % time)
        kc = int(os.environ.get("FPM_AFAU_SPLIT_TERMS", "2")) * HD if split else (kx(1, HD) if x3 else HD)
        ops.gemm(att, wp["row_Wc"], B * n1max, E, kc, att.shape[1], att.shape[1], bias=wp["row_bc"], out_f=mh, ldc=E)
        g_row = self._afau_block(wp, "row", B, n1max, mh=mh)
        if col is None or col[2] != n2max:
            col = self._afau_col(wp, bt)
        n2u, gm_u, _ = col
        n2c = bt.n_host[1].numpy()
        inv = np.searchsorted(n2u, n2c) if len(n2u) != len(n2c) or not np.array_equal(n2u, n2c) else None
        g_col = gm_u if inv is None else gm_u.index_select(0, torch.as_tensor(inv, dtype=torch.long).to(
            dev, non_blocking=True))
        ks = torch.empty(B, device=dev, dtype=torch.float32)
        ops.afau_head(g_row, g_col, B, E, wp["final_row0w"], wp["final_row0b"], wp["final_row2w"],
                      wp["final_row2b"], wp["final_col0w"], wp["final_col0b"], wp["final_col2w"], wp["final_col2b"], ks)
        return ks

    def _mark(self, name):
        """Diagnostic stage timing (FPM_STAGE_TIMING=1): synchronises, so never in timed runs."""
        if self._stage_timing:
            torch.cuda.synchronize()
            t = time.perf_counter()
            self.stage_times[name] = self.stage_times.get(name, 0.0) + (t - self._t_last)
            self._t_last = t

    def _edge_affinity(self, wp, bt, gw, f1, f2):
        """Ke[b] = 0.5 * (softplus((Xe1 o c') Xe2^T) - 0.5), Xe = x'[src] - x'[dst] from the
        SplineConv output (ngm.py:250-289; affinity_layer.py:11-19) -> (B, E1max, E2max) fp32,
        zero outside each pair's E1 x E2 block."""
        dev = bt.device
        B, D = bt.B, C.NODE_FEATURE_DIM
        ce = torch.empty(B, D, device=dev, dtype=torch.float32)
        ops.gemm(gw, wp["eaff_w"], B, D, C.GLOBAL_STATE_DIM, C.GLOBAL_STATE_DIM, C.GLOBAL_STATE_DIM,
                 epi=ops.EPI_TANH, bias=wp["eaff_b"], out_f=ce)
        xe, cnt = [], []
        for side, f in ((0, f1), (1, f2)):
            off = torch.as_tensor(bt.edge_off[side], dtype=torch.long)
            c = off[1:] - off[:-1]
            emax = max(int(c.max()), 1)
            pair = torch.repeat_interleave(torch.arange(B), c)
            row = pair * emax + (torch.arange(int(off[-1])) - off[pair])
            x = ops.edge_diff_padded(f, bt.src[side], bt.dst[side], pair.to(dev, torch.int32),
                                     row.to(dev, torch.int32), B * emax, cscale=ce if side == 0 else None)
            xe.append((x, emax))
            cnt.append(c.to(dev, torch.int32))
        (x1, e1), (x2, e2) = xe
        Ke = torch.empty(B, e1, e2, device=dev, dtype=torch.float32)
        ops.gemm(x1, x2, e1, e2, D, D, D, batch=B, sA=e1 * D, sB=e2 * D, epi=ops.EPI_HALF_AFFINITY, out_f=Ke,
                 ldc=e2, sC=e1 * e2, n1=cnt[1], n2=cnt[0])
        return Ke

    def global_coef(self, bt):
        """Global weights w = L2norm(cat(w1, w2)) and vertex-affinity coefficients c = tanh(A w + a)
        for every pair of ``bt`` (ngm.py:262-268, affinity_layer.py:13); one launch per forward."""
        wp = self.packed(bt.device)
        gw = ops.global_weights(bt.w[0], bt.w[1])
        coef = torch.empty(bt.B, C.NODE_FEATURE_DIM, device=bt.device, dtype=torch.float32)
        ops.gemm(gw, wp["aff_w"], bt.B, C.NODE_FEATURE_DIM, C.GLOBAL_STATE_DIM, C.GLOBAL_STATE_DIM,
                 C.GLOBAL_STATE_DIM, epi=ops.EPI_TANH, bias=wp["aff_b"], out_f=coef)
        return gw, coef

    def run_gpu_stage(self, bt, keep_feats=False, s_out=None, ss_out=None, gc=None, x_ops=(None, None)):
        """Everything up to ds_mat on the GPU.  Returns a dict of device tensors.  ``gc``: this
        batch's rows of global_coef() when computed for a parent batch; ``x_ops``: its rows of the
        parent's bf16 operand copies of the node features (cast once per forward)."""
        keep_feats = keep_feats or self.compute_ke
        self._keep_feats = keep_feats
        if self._stage_timing:
            torch.cuda.synchronize()
            self._t_last = time.perf_counter()
        wp = self.packed(bt.device)
        dev = bt.device
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        N = n1max * n2max
        gw, coef = gc if gc is not None else self.global_coef(bt)
        self._mark("coef")
        plan0, x1c, f1 = self._spline_side(wp, bt, 0, coef, x_ops[0])
        plan1, x2, f2 = self._spline_side(wp, bt, 1, None, x_ops[1])
        self._mark("splineconv")
        if self._offset_events is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self._offset_events.append(ev)
        # Kp^T per pair: emb0[b][j][i] = softplus((x1_i o c) . x2_j) - 0.5 on the valid block (ngm.py:277-321)
        X = torch.empty(B, 1, n2max, n1max, device=dev, dtype=torch.float32)
        ops.gemm(x2, x1c, n2max, n1max, C.NODE_FEATURE_DIM, C.NODE_FEATURE_DIM, C.NODE_FEATURE_DIM, batch=B,
                 sA=n2max * C.NODE_FEATURE_DIM, sB=n1max * C.NODE_FEATURE_DIM, epi=ops.EPI_AFFINITY, out_f=X,
                 ldc=n1max, sC=N, n1=bt.n1, n2=bt.n2)
        Kp = X
        Ke = self._edge_affinity(wp, bt, gw, f1, f2) if self.compute_ke else None
        self._mark("affinity")
        csr1 = ops.plan_csr(plan0, bt.E[0], B * n1max)
        csr2 = ops.plan_csr(plan1, bt.E[1], B * n2max)
        zbuf = torch.empty(B, n2max, n1max, device=dev, dtype=torch.float32)
        vpart = torch.empty(B, n2max, n1max, device=dev, dtype=torch.float32)
        Cin = 1
        for l in range(C.GNN_LAYER):
            Xn = torch.empty(B, 17, n2max, n1max, device=dev, dtype=torch.float32)
            last = l == C.GNN_LAYER - 1      # fuse the final classifier's x1 part (ngm.py:368)
            ops.gnn_layer(X, Cin, B, n1max, n2max, csr1, csr2, bt.n1, bt.n2, wp["gnn%d" % l], Xn, zbuf,
                          vpart=vpart if last else None, cls_w=wp["cls_w"] if last else None)
            # Sinkhorn(20, tau) on Z[i][j] = z[j*n1max + i], written into channel 16 (gnn.py:217-222)
            ops.sinkhorn(zbuf.transpose(1, 2), bt.n1, bt.n2, C.GNN_SK_ITER, self.tau, True,
                         out=Xn[:, 16].transpose(1, 2))
            X, Cin = Xn, 17
            self._mark("gnn%d" % l)
        s = s_out if s_out is not None else torch.empty(B, n1max, n2max, device=dev, dtype=torch.float32)
        ops.node_classifier(X, B, n1max, n2max, wp["cls_w"], wp["cls_b"], s, vpart=vpart)
        ss = ops.sinkhorn(s, bt.n1, bt.n2, C.SK_ITER_NUM, self.tau, True, out=ss_out)
        self._mark("final_sinkhorn")
        out = dict(s=s, ss=ss, Kp=Kp[:, 0].transpose(1, 2), coef=coef)
        if keep_feats:
            out["feat0"], out["feat1"] = f1, f2
        if Ke is not None:
            out["Ke"] = Ke
        return out

    # ------------------------------------------------------------------------------------------
    def _streams(self, dev):
        key = str(dev)
        if key not in self._stream_cache:
            # FPM_STREAM_PRIO=1: compute streams at high priority (the ds_mat copy stream stays at
            # the default) -- A/B switch for the copy blit's interference
            prio = -1 if os.environ.get("FPM_STREAM_PRIO", "0") == "1" else 0
            self._stream_cache[key] = [torch.cuda.Stream(dev, priority=prio) for _ in range(self.n_streams)]
        return self._stream_cache[key]

    def _lsa_streams(self, dev):
        key = "lsa:" + str(dev)
        if key not in self._stream_cache:
            self._stream_cache[key] = [torch.cuda.Stream(dev) for _ in range(2)]
        return self._stream_cache[key]

    def pipeline_chunks(self, B):
        """Sub-batches per forward so the host Hungarian of chunk c overlaps the GPU work of c+1."""
        if self.chunks is not None:
            return max(1, min(self.chunks, B))
        if os.environ.get("FPM_CHUNKS"):
            return max(1, min(int(os.environ["FPM_CHUNKS"]), B))
        return max(1, min(8, B // 128))

    def _enqueue_copy(self, dev, b0, b1, o, done, after=None):
        """ds_mat[b0:b1] -> pinned host memory on the copy stream once ``done`` (and ``after``, if
        given) have fired; returns the copy's completion event."""
        cs = self._copy_stream(dev)
        cs.wait_event(done)
        if after is not None:
            cs.wait_event(after)
        with torch.cuda.stream(cs):
            if self.copy_kind > 0:
                ops.memcpy_async(self._pinned[b0:b1], o["ds_mat"][b0:b1], self.copy_kind)
            elif self.copy_blocks > 0:
                ops.copy_async(self._pinned[b0:b1], o["ds_mat"][b0:b1], self.copy_blocks)
            else:
                self._pinned[b0:b1].copy_(o["ds_mat"][b0:b1], non_blocking=True)
        ev = torch.cuda.Event(enable_timing=True, blocking=self.blocking_wait)
        ev.record(cs)
        return ev

    def _stage_a(self, part, b0, b1, o, keep_feats, gt_ks, min_pt, st, gc, col=None, defer=None, xop=None):
        """GPU stage of one chunk (on its stream): everything up to ds_mat, then its D2H copy."""
        dev = part.device
        x_ops = tuple(None if t is None else t[b0 * part.nmax[s]:b1 * part.nmax[s]]
                      for s, t in enumerate(xop or (None, None)))
        r = self.run_gpu_stage(part, keep_feats, s_out=o["s"][b0:b1], ss_out=o["ss"][b0:b1],
                               gc=(gc[0][b0:b1], gc[1][b0:b1]), x_ops=x_ops)
        ks = o["k_prob"][b0:b1]
        if self.regression:
            ks.copy_(self._afau(self.packed(dev), o["ss"][b0:b1], part, col=col))
        else:
            ks.copy_(gt_ks[b0:b1] / min_pt[b0:b1])
        self._mark("afau")
        k_used = gt_ks[b0:b1] if self.training else ks * min_pt[b0:b1]
        ops.soft_topk_fwd(o["ss"][b0:b1], part.n1, part.n2, k_used.contiguous(), C.SK_ITER_NUM, self.tau,
                      out=o["ds_mat"][b0:b1], steps=o["sk_steps"][b0:b1],
                      out_host=self._pinned[b0:b1] if self.zero_copy else None)
        o["_kk"][b0:b1].copy_(ks * min_pt[b0:b1])
        self._mark("soft_topk")
        if self.lsa_mode == "device":
            # the Hungarian kernel is latency-bound (one wave per pair): run it and the selection /
            # classifier on a side stream so the next chunks' GPU stages are not queued behind it
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(st)
            self._lsa_rr = getattr(self, "_lsa_rr", 0) + 1
            side = self._lsa_streams(dev)[self._lsa_rr % 2]
            side.wait_event(ev)
            with torch.cuda.stream(side):
                self._stage_c_device(part, b0, b1, o)
            return r, ev
        if not self.zero_copy and self.copy_stream:
            # the D2H copy is a blit kernel: on a stream of its own it does not hold back the next
            # chunk queued on this compute stream
            done = torch.cuda.Event()
            done.record(st)
            if defer is not None:
                defer.append((b0, b1, done))
                return r, None
            return r, self._enqueue_copy(dev, b0, b1, o, done)
        if not self.zero_copy:
            self._pinned[b0:b1].copy_(o["ds_mat"][b0:b1], non_blocking=True)
        ev = torch.cuda.Event(enable_timing=True, blocking=self.blocking_wait)
        ev.record(st)
        return r, ev

    def _copy_stream(self, dev):
        key = "copy:" + str(dev)
        if key not in self._stream_cache:
            self._stream_cache[key] = torch.cuda.Stream(dev)
        return self._stream_cache[key]

    def _stage_c_device(self, part, b0, b1, o):
        """Device Hungarian + greedy selection + MatchClassifier of one chunk, queued on the
        chunk's stream right behind its soft top-k (no host round trip)."""
        wp = self._pack
        assign, status = ops.lsa_batch_device(o["ds_mat"][b0:b1], part.n1, part.n2,
                                              status=o["_lsa_status"][b0:b1])
        ops.topk_select(o["ds_mat"][b0:b1], assign, o["_kk"][b0:b1], lsa_out=o["lsa"][b0:b1],
                        out=o["perm_mat"][b0:b1])
        ops.match_cls(o["s"][b0:b1], o["perm_mat"][b0:b1], wp["mc_w1"], wp["mc_b1"], wp["mc_sc1"], wp["mc_sh1"],
                      wp["mc_w2"], wp["mc_b2"], wp["mc_sc2"], wp["mc_sh2"], wp["mc_fcw"], wp["mc_fcb"],
                      logits=o["cls_logits"][b0:b1], prob=o["cls_prob"][b0:b1],
                      dtype=ops.BF16 if self.dtype_mode == "bf16" else ops.F32)

    def _stage_c(self, part, b0, b1, o):
        """Host Hungarian (utils/hungarian.py: LSA of -ds_mat per pair) + greedy selection +
        MatchClassifier of one chunk; the caller waits for the chunk's D2H event first."""
        dev = part.device
        wp = self._pack
        t = time.perf_counter()
        assign = ops.lsa_batch_host(self._pinned[b0:b1], part.n_host[0], part.n_host[1], self.lsa_threads)
        dt = time.perf_counter() - t
        assign_d = assign.to(dev, non_blocking=True)
        ops.topk_select(o["ds_mat"][b0:b1], assign_d, o["_kk"][b0:b1], lsa_out=o["lsa"][b0:b1],
                        out=o["perm_mat"][b0:b1])
        self._mark("lsa+h2d+select")
        ops.match_cls(o["s"][b0:b1], o["perm_mat"][b0:b1], wp["mc_w1"], wp["mc_b1"], wp["mc_sc1"], wp["mc_sh1"],
                      wp["mc_w2"], wp["mc_b2"], wp["mc_sc2"], wp["mc_sh2"], wp["mc_fcw"], wp["mc_fcb"],
                      logits=o["cls_logits"][b0:b1], prob=o["cls_prob"][b0:b1],
                      dtype=ops.BF16 if self.dtype_mode == "bf16" else ops.F32)
        self._mark("match_cls")
        return dt

    def run(self, bt, gt_perm=None, label=None, keep_feats=False, chunks=None):
        """Full forward, pipelined over sub-batches ("chunks").  Every chunk's GPU stage is queued
        at once, alternating over two streams (per-pair kernels of neighbouring chunks -- Sinkhorn,
        soft top-k, AFA-U, one workgroup per pair -- then fill the 256 CUs together); the host LSA
        of chunk c starts as soon as its ds_mat lands in pinned memory while the GPU continues;
        chunk c's selection + classifier follow its LSA on its stream."""
        dev = bt.device
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        K = chunks if chunks is not None else self.pipeline_chunks(B)
        if self.compute_ke:
            K = 1          # Ke blocks are padded to per-chunk edge maxima: keep one chunk
        parts = bt.split(K, self.tail_splits if K > 1 else 0, self.head_splits if K > 1 else 0)
        t0 = time.perf_counter()
        min_pt = torch.minimum(bt.n1, bt.n2).to(torch.float32)
        if gt_perm is None:
            gt_ks = min_pt.clone()     # synthetic pairs: identity ground truth
        else:
            gt_ks = torch.as_tensor(gt_perm).to(dev).reshape(B, -1).sum(-1).to(torch.float32)
        f32 = dict(device=dev, dtype=torch.float32)
        o = {k: torch.empty(B, n1max, n2max, **f32) for k in ("s", "ss", "ds_mat", "perm_mat", "lsa")}
        o.update({k: torch.empty(B, **f32) for k in ("k_prob", "cls_logits", "cls_prob", "_kk")})
        o["sk_steps"] = torch.empty(B, device=dev, dtype=torch.int32)
        o["_lsa_status"] = torch.zeros(B, device=dev, dtype=torch.int32)
        device_lsa = self.lsa_mode == "device"
        if not device_lsa and (self._pinned is None or self._pinned.shape != o["ds_mat"].shape):
            self._pinned = torch.empty(o["ds_mat"].shape, dtype=torch.float32, pin_memory=True)
        main = torch.cuda.current_stream(dev)
        ev_start = torch.cuda.Event(enable_timing=True)
        ev_start.record(main)
        gc = self.global_coef(bt)
        # bf16 operand rows of both sides' node features in one launch each, before any chunk's
        # ds_mat D2H is in flight (cast per chunk, they ran beside the copy's blit kernel and
        # stalled ~14x; a shared probe side is cast inside its chunk's one-graph SplineConv)
        xop = None
        if self.dtype_mode == "bf16" and len(parts) > 1:
            xop = tuple(None if (s == 0 and bt.shared0) else ops.cast_bf16(bt.x[s]) for s in range(2))
        # the AFA-U column block once for the whole batch (per distinct n2), before the chunks
        col = (self._afau_col(self.packed(dev), bt)
               if self.regression and os.environ.get("FPM_AFAU_COLDEDUP", "1") == "1"
               and os.environ.get("FPM_AFAU_COLFWD", "1") == "1" else None)
        ev_coef = torch.cuda.Event()
        ev_coef.record(main)
        streams = self._streams(dev) if (len(parts) > 1 and self.n_streams > 1) else [main]
        for st in streams:
            if st is not main:
                st.wait_event(ev_coef)
        outs, events = [], []
        lag = 2 if (self.copy_defer and len(parts) > 2 and len(streams) == 2 and self.copy_stream
                    and not self.zero_copy and not device_lsa) else 0
        pending = [] if lag else None
        self._plan_events = [] if lag else None
        self._offset_events = [] if (self.stream_offset and len(streams) == 2 and len(parts) > 1) else None
        try:
            for c, part in enumerate(parts):
                st = streams[c % len(streams)]
                b0, b1 = (0, B) if part is bt else part.pair_range     # a chunk's range inside bt
                if c == 1 and self._offset_events:
                    st.wait_event(self._offset_events[0])
                    self._offset_events = None
                with torch.cuda.stream(st):
                    r, ev = self._stage_a(part, b0, b1, o, keep_feats, gt_ks, min_pt, st, gc, col=col, defer=pending,
                                          xop=xop)
                outs.append(r)
                events.append(ev)
                if lag and c >= lag:
                    # chunk c - lag's copy after chunk c's first plan (same stream as chunk c - lag)
                    pb0, pb1, pdone = pending[c - lag]
                    events[c - lag] = self._enqueue_copy(dev, pb0, pb1, o, pdone, after=self._plan_events[c])
            if lag:
                for c in range(max(0, len(parts) - lag), len(parts)):
                    pb0, pb1, pdone = pending[c]
                    events[c] = self._enqueue_copy(dev, pb0, pb1, o, pdone)
        finally:
            self._plan_events = None
            self._offset_events = None
        t_enq = time.perf_counter()
        t_lsa, t_first = 0.0, None
        for c, (part, ev) in enumerate(zip(parts, events)):
            if device_lsa:
                break
            b0, b1 = (0, B) if part is bt else part.pair_range     # a chunk's range inside bt
            ev.synchronize()
            t_first = t_first or time.perf_counter()
            with torch.cuda.stream(streams[c % len(streams)]):
                t_lsa += self._stage_c(part, b0, b1, o)
        for st in streams:
            if st is not main:
                main.wait_stream(st)
        if device_lsa:
            for st in self._lsa_streams(dev):
                main.wait_stream(st)
            bad = torch.nonzero(o["_lsa_status"]).view(-1)
            if bad.numel():
                raise RuntimeError("hungarian: pair %d is infeasible or has NaN/-inf costs" % int(bad[0]))
        res = {k: v for k, v in o.items() if not k.startswith("_")}
        if len(outs) == 1 or keep_feats:
            for k in outs[0]:
                if k not in ("s", "ss"):
                    res[k] = outs[0][k] if len(outs) == 1 else torch.cat([r[k] for r in outs])
        ks, logits = o["k_prob"], o["cls_logits"]
        if label is not None:
            res["cls_loss"] = F.binary_cross_entropy_with_logits(logits, torch.as_tensor(label).to(dev).view(-1).float())
        else:
            res["cls_loss"] = torch.tensor(0.0, device=dev)
        if self.regression:
            res["ks_loss"] = F.mse_loss(ks, gt_ks / min_pt) * self.k_factor
            res["ks_error"] = F.l1_loss(ks * min_pt, gt_ks)
        else:
            res["ks_loss"] = 0.0
            res["ks_error"] = 0.0
        # GPU time of the stages before the Hungarian (all chunks), from events on the streams
        self.last_timing = dict(gpu_stage_s=ev_start.elapsed_time(events[-1]) / 1e3, lsa_s=t_lsa,
                                first_chunk_wait_s=(t_first or t0) - t0, chunks=len(parts),
                                enqueue_s=t_enq - t0, total_s=time.perf_counter() - t0)
        return res

    def image_features(self, images, Ps, ns, dev=None):
        """ngm.py:226-248 on the device: per side, node_layers/edge_layers (ResNet-18 convolutions
        on MIOpen, channels_last; bf16 autocast in the bf16 mode), then one HIP kernel set for
        global max-pool + channel L2-norm + bilinear feature_align + [U || F] concat.
        Returns (node feature rows 2 x (B*nmax, 768) with zero padding rows, globals 2 x (B, 512))."""
        if not hasattr(self, "node_layers"):
            raise NotImplementedError("image input needs the backbone: this Net was built with backbone=False "
                                      "(pass data_dict['node_features'] / ['global_features'] instead)")
        dev = dev or torch.device("cuda", torch.cuda.current_device())
        if self._backbone_dev != dev:
            for m in (self.node_layers, self.edge_layers):
                m.to(device=dev, memory_format=torch.channels_last)
            self._backbone_dev = dev
        xs, gs = [], []
        # train mode with autograd on (train.py): the backbone runs under autograd and the align
        # stage has its HIP backward (fpm.train.FeatureAlignFn); inference: no graph
        grad = self.training and torch.is_grad_enabled()
        for img, pts, n in zip(images, Ps, ns):
            img = torch.as_tensor(img)
            if img.dim() == 3:
                img = img.unsqueeze(0)
            img = img.to(device=dev, dtype=torch.float32).contiguous(memory_format=torch.channels_last)
            with torch.set_grad_enabled(grad), torch.autocast("cuda", dtype=torch.bfloat16,
                                                               enabled=self.dtype_mode == "bf16"):
                nodes = self.node_layers(img)
                edges = self.edge_layers(nodes)
            pts = torch.as_tensor(pts).to(device=dev, dtype=torch.float32)
            n32 = torch.as_tensor(n).view(-1).to(device=dev, dtype=torch.int32)
            if grad:
                from .train import FeatureAlignFn
                x, g = FeatureAlignFn.apply(nodes.float(), edges.float(), pts.contiguous(), n32, C.RESCALE)
            else:
                x, g = ops.feature_align(nodes.float(), edges.float(), pts, n32, ori_size=C.RESCALE)
            xs.append(x)
            gs.append(g)
        return xs, gs

    def _batch_from_dict(self, data_dict, dev):
        dd = data_dict
        if "node_features" not in dd and "images" in dd:
            xs, gs = self.image_features(dd["images"], dd["Ps"], dd["ns"], dev)
            dd = dict(dd)
            dd["node_features"] = [x.view(int(torch.as_tensor(p).shape[0]), int(torch.as_tensor(p).shape[1]), -1)
                                   for x, p in zip(xs, dd["Ps"])]
            dd["global_features"] = gs
        if "pyg_graphs" not in dd and "Ps" in dd and "node_features" in dd:
            # graphs as GMDataset builds them ('tri', gmdataset.py:233-244), on the device
            nf = [torch.as_tensor(t) for t in dd["node_features"]]
            Ps = [torch.as_tensor(p).to(device=dev, dtype=torch.float32) for p in dd["Ps"]]
            if any(t.dim() != 3 for t in nf):
                raise ValueError("device graph build needs padded (B, nmax, 768) node_features")
            x = []
            for t, n in zip(nf, dd["ns"]):
                t = t.to(device=dev, dtype=torch.float32)
                keep = torch.arange(t.shape[1], device=dev)[None, :] < torch.as_tensor(n).to(dev).view(-1, 1)
                x.append(torch.where(keep[..., None], t, torch.zeros((), device=dev)).reshape(-1, t.shape[-1]).contiguous())
            w = [torch.as_tensor(t).to(device=dev, dtype=torch.float32).contiguous() for t in dd["global_features"]]
            return DeviceBatch.from_keypoints(Ps, [torch.as_tensor(n).view(-1) for n in dd["ns"]], x, w, dev)
        return DeviceBatch.from_data_dict(dd, dev)

    def forward(self, data_dict, regression=True):
        """Reference signature (ngm.py:205).  ``regression`` is accepted and ignored there too."""
        dev = torch.device("cuda", torch.cuda.current_device())
        bt = data_dict.get("fpm_batch")
        if bt is None:
            bt = self._batch_from_dict(data_dict, dev)
        gt = data_dict.get("gt_perm_mat")
        if self.training and torch.is_grad_enabled():
            # train.py / training_loop.py: differentiable forward, hand-written HIP backward (fpm.train)
            from .train import run_train
            res = run_train(self, bt, gt_perm=gt, label=data_dict.get("label"))
        else:
            res = self.run(bt, gt_perm=gt, label=data_dict.get("label"))
        self.last_outputs = res          # all outputs incl. intermediates (s, ss, ...) for inspection
        data_dict.update({
            "ds_mat": res["ds_mat"],
            "perm_mat": res["perm_mat"],
            "ks_loss": res["ks_loss"],
            "ks_error": res["ks_error"],
            "cls_loss": res["cls_loss"],
            "cls_prob": res["cls_prob"],
            "k_prob": res["k_prob"],
        })
        return data_dict
