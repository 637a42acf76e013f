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


def rank_cpu_set(local_rank, local_world, aff=None):
    """The CPUs of the node-local rank ``local_rank`` of ``local_world``: a contiguous, disjoint slice
    of the (sorted) affinity mask, at least one CPU each (ranks share CPUs round-robin only when the
    mask has fewer CPUs than ranks)."""
    cpus = sorted(aff if aff is not None else os.sched_getaffinity(0))
    local_world = max(1, int(local_world))
    if len(cpus) < local_world:
        return [cpus[int(local_rank) % len(cpus)]]
    k = len(cpus) // local_world
    return cpus[int(local_rank) * k:(int(local_rank) + 1) * k]


def pin_rank_cpus():
    """Under torch.distributed.run with several ranks on the node: restrict this process to its own
    slice of the affinity mask (rank_cpu_set), so the ranks' host Hungarian pools do not compete for
    the same cores (FPM_PIN_RANKS=0: off).  Returns the CPU list or None."""
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    if lws <= 1 or os.environ.get("FPM_PIN_RANKS", "1") == "0" or os.environ.get("FPM_RANK_PINNED") == "1":
        return None
    cpus = rank_cpu_set(int(os.environ.get("LOCAL_RANK", "0")), lws)
    os.sched_setaffinity(0, cpus)
    os.environ["FPM_RANK_PINNED"] = "1"
    return cpus


def host_cpu_share():
    """CPUs this process may use for the host Hungarian pool.  ``FPM_CPU_SHARE`` sets it explicitly
    (``FPM_LSA_THREADS`` sets the pool size itself, default 4 per CPU of the share).  Otherwise:
    OMP_NUM_THREADS (16 per GPU on the pool) capped by the affinity mask; under
    torch.distributed.run (LOCAL_WORLD_SIZE > 1) the cap is this rank's slice of the mask
    (rank_cpu_set; after pin_rank_cpus the mask IS the slice), and a share of 1 is read as the
    launcher's OMP_NUM_THREADS=1 default (it exports it when the variable was unset) and replaced
    by the slice (at most 16) -- set FPM_CPU_SHARE=1 to really run on one CPU."""
    n_aff = len(os.sched_getaffinity(0))
    if os.environ.get("FPM_CPU_SHARE"):
        return max(1, min(int(os.environ["FPM_CPU_SHARE"]), n_aff))
    omp = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1) if "LOCAL_WORLD_SIZE" in os.environ else 0
    if lws >= 1:
        cap = n_aff if os.environ.get("FPM_RANK_PINNED") == "1" else len(
            rank_cpu_set(int(os.environ.get("LOCAL_RANK", "0")), lws))
        if omp <= 1:
            omp = 16
        return max(1, min(omp, cap))
    return max(1, min(omp, n_aff))


class _Node(nn.Module):
    pass


class _SharedProbe:
    """Probe x gallery: the shared side-0 graph's two SplineConv layers (fp32 rows of one graph),
    computed once per forward in the prologue and handed to every chunk in place of its side-0
    operand rows (chunk slicing leaves it whole)."""

    def __init__(self, y):
        self.y = y


class _TailView:
    """Pairs [r0, r1) of a (sub-)batch ``part`` for the tail stages (AFA-U, soft top-k, Hungarian,
    selection, classifier): device views of the pair sizes, no copies; ``pair_range`` is its range in
    the forward's batch."""

    def __init__(self, part, r0, r1, pair_range):
        self.B = r1 - r0
        self.device = part.device
        self.nmax = part.nmax
        self.n = [part.n[0][r0:r1], part.n[1][r0:r1]]
        self.n_host = [part.n_host[0][r0:r1], part.n_host[1][r0:r1]]
        self.pair_range = pair_range

    n1 = property(lambda self: self.n[0])
    n2 = property(lambda self: self.n[1])
    n1max = property(lambda self: self.nmax[0])
    n2max = property(lambda self: self.nmax[1])


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
                 backbone=True, lsa=None, afau=None):
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
        # AFA-U operands in the bf16 mode (``afau`` argument, else FPM_AFAU_DTYPE): "bf16x3"
        # (default) every AFA-U product on split near-fp32 operands ([hi | lo | hi] x [W_hi | W_hi |
        # W_lo], written by the producing kernels' epilogues): with the bf16 SplineConv / affinity it
        # stays within the north star's 1e-4 fp32 gate on ss / ds_mat / k_prob (gated_probe: k_prob
        # 3.0e-5 from the fp32 oracle at C3); "bf16s" the combine product on split operands, FFN on
        # plain bf16 (k_prob 3.9-7.7e-4); "bf16" the attention output rounded to bf16 too (8e-3);
        # "f32" fp32 AFA-U products.
        self.afau_mode = "f32" if dtype == "f32" else (afau or os.environ.get("FPM_AFAU_DTYPE", "bf16x3"))
        if self.afau_mode not in ("f32", "bf16", "bf16s", "bf16x3"):
            raise ValueError("afau / FPM_AFAU_DTYPE must be f32, bf16, bf16s or bf16x3")
        # Hungarian pool: 4 threads per CPU of the process's share (FPM_LSA_THREADS overrides).  Measured
        # on the 16-CPU box share: 16 / 32 / 48 threads -> 29-44 / 17-22 / 17-18 ms per 1024 pairs
        # (the pairs of a chunk differ in cost; idle stragglers at each chunk's join dominate at 1x).
        # The threads stay inside the share (its affinity mask); more threads than CPUs only let a
        # tail group's pairs all start at once and share the cores evenly, so the group ends when its
        # total work does rather than behind a straggler.  Round 6 (profiles/r06_lsa_threads_ab.txt):
        # 64 vs 32 threads +5 % on the 128-pair forward (21.8-22.0 vs 20.2-21.0 K), C3 equal.
        share = host_cpu_share()
        self.lsa_threads = lsa_threads or int(os.environ.get("FPM_LSA_THREADS", str(4 * share)))
        self.chunks = chunks
        # quadratic (edge) affinity Ke (ngm.py:282-289): dead for every output, off by default
        self.compute_ke = compute_ke
        self._pack = None
        self._pack_key = None
        self._pack_gen = 0
        self._pinned = None
        self._stream_cache = {}
        # FPM_STREAMS: compute streams of the chunk pipeline (1 = single-stream profiling runs)
        self.n_streams = max(1, int(os.environ.get("FPM_STREAMS", "2")))
        # the last chunk halved this many times: the two streams' last chunks land together, so the
        # host Hungarian's tail after the GPU is their (short) LSA
        self.tail_splits = int(os.environ.get("FPM_TAIL", "2"))
        # one-chunk forwards (small per-GPU batches, e.g. 128 pairs = BASELINE's 1024 over 8 GPUs):
        # the tail after ss (AFA-U, soft top-k, ds_mat D2H) runs in FPM_TAIL_GROUPS pair groups of at
        # least FPM_TAIL_MIN pairs, so the host Hungarian of the first group starts while the GPU
        # still works on the others (1 = off)
        self.tail_groups = max(1, int(os.environ.get("FPM_TAIL_GROUPS", "4")))
        self.tail_min = max(1, int(os.environ.get("FPM_TAIL_MIN", "16")))
        self.tail_last = float(os.environ.get("FPM_TAIL_LAST", "0.5"))
        # FPM_TAIL_STREAMS (2): the tail groups alternate between the forward's stream and the (idle in
        # one-chunk forwards) second chunk stream, so one group's latency-bound kernels (soft top-k,
        # the attention: one workgroup per pair) run beside the next group's; 1 = one stream
        # (3 / 4: further streams of their own join the rotation)
        self.tail_streams = max(1, min(4, int(os.environ.get("FPM_TAIL_STREAMS", "2"))))
        # defer each chunk's ds_mat D2H until the spline plans of the chunk queued two places later
        # (same compute stream) have run: those latency-bound kernels otherwise run beside the
        # copy's blit kernel and stall ~10x
        self.copy_defer = int(os.environ.get("FPM_COPY_DEFER", "1"))
        if self.copy_defer not in (0, 1):
            raise ValueError("FPM_COPY_DEFER must be 0 or 1")
        # FPM_LSA_ASYNC=1: chunks' Hungarian batches queue on persistent workers that serve pairs
        # first-in first-out across chunks (a chunk's pairs start while the previous chunk's slowest
        # pairs still run) instead of one blocking batch per chunk
        self.lsa_async = os.environ.get("FPM_LSA_ASYNC", "1") != "0"
        self._enqueue_lock = None      # set by fpm.parallel.ShardedNet (one lock for its replicas)
        # FPM_AFAU_FUSE=0: the AFA-U block's FFN output through HBM + a separate instance norm (A/B)
        self.afau_fuse_norm = os.environ.get("FPM_AFAU_FUSE", "1") != "0"
        # FPM_GRAPHS=1: multi-chunk inference forwards replay HIP graphs captured per (batch, chunk)
        # (host enqueue 8 -> 1 ms per 1024 pairs; the GPU stage measured 4 % slower than eager
        # launches, so off by default; fpm.parallel.ShardedNet turns it on); see run()
        self.use_graphs = os.environ.get("FPM_GRAPHS", "0") == "1"
        # ds_mat for the host Hungarian written to pinned memory by the soft top-k kernel itself
        # (zero-copy) instead of a blit-kernel D2H: 0 off, 1 one-chunk tail groups, 2 every chunk
        self.zero_copy = int(os.environ.get("FPM_ZERO_COPY", "0"))
        # FPM_STAGEC_STREAM=1: stage C (selection + classifier) on the main stream as soon as each unit's
        # Hungarian finishes, instead of on its chunk's stream behind the later chunks: measured 2-3 %
        # SLOWER GPU stage at C3 (the 128-pair selection / classifier kernels co-running with the
        # pipeline) with no shorter end of the forward (the last units' Hungarian sets it), round 5;
        # off by default
        self.stagec_stream = os.environ.get("FPM_STAGEC_STREAM", "0") == "1"
        # the prologue's casts + AFA-U column block beside its plans + coefficients (FPM_PROLOGUE_FORK=0: serial)
        self.prologue_fork = os.environ.get("FPM_PROLOGUE_FORK", "1") != "0"
        # bf16 mode: the vertex affinity Kp on split near-fp32 operands (FPM_KP_X3=0: plain bf16 rows).
        # Kp feeds the tau = 0.01 Sinkhorns of the GNN layers directly; its bf16 rounding was the
        # largest bf16-mode source of k_prob deviation (tools/kprob_diag.py)
        self.kp_x3 = os.environ.get("FPM_KP_X3", "1") != "0"
        # bf16 mode, small graphs: batches whose padded box is at most FPM_SC_F32_NMAX (64) keypoints run
        # the SplineConv products and the vertex affinity in fp32 (a few percent of such a forward's
        # time).  The bf16 products round x, W and the stored product rows to bf16 (relative 2^-9
        # each); on ill-conditioned image-derived pairs that moved k_prob by up to ~1e-4 beyond the
        # fp32 reference's own deviation (tools/kprob_yround.py), so the bf16 mode keeps them for the
        # large graphs where they pay (C3: n = 256) and stays near-fp32 below.
        self.sc_f32_nmax = int(os.environ.get("FPM_SC_F32_NMAX", "64"))
        # the k chain in fp64 (csrc/precise.hip): batches whose padded box is at most FPM_K_F64_NMAX
        # (64, at most 128) keypoints run everything after Kp -- the three GNN layers with their
        # Sinkhorns, the readout, the final Sinkhorn and the AFA-U regressor -- in fp64, both modes,
        # inference only.  On image-derived pairs of that size k_prob is ill-conditioned: the fp32
        # rounding of any one stage after Kp moves it by up to ~6e-5 and the fp32 reference sits up
        # to 2e-4 from its own fp64 value (tools/kprob_arith.py); in fp64 the device lands within
        # ~5e-6 of it.  0 = off.
        self.k_f64_nmax = min(128, int(os.environ.get("FPM_K_F64_NMAX", "64")))
        # FPM_PROLOGUE_GRAPH: the eager forward's prologue (coefficients, casts, AFA-U column block,
        # spline plans: ~15 small launches whose Python enqueue left the GPU idle ~0.5 ms at the start
        # of a 128-pair forward) replayed from a HIP graph captured on the batch's first forward.
        # 1 (default): one-chunk forwards only -- the 128-pair share line 18.6-19.0 K -> 19.9-20.0 K
        # pairs/s, while multi-chunk C3 forwards measured 1.8 % slower with it (29.8-29.9 vs 30.3-30.6 K,
        # round 5: the replay's extra hardware queue beside the two chunk streams); 2: every forward
        self.prologue_graph = int(os.environ.get("FPM_PROLOGUE_GRAPH", "1"))
        self._gstate = None
        self._pgstate = None
        self._keep_feats = False
        self._stage_timing = os.environ.get("FPM_STAGE_TIMING", "0") == "1"
        self._stage_events = os.environ.get("FPM_STAGE_EVENTS", "0") == "1"
        self._ev_marks = []
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
            wf = torch.cat([sd[pre + ".weight"].to(device).transpose(1, 2),
                            sd[pre + ".root"].to(device).t()[None]]).contiguous().float()
            d["W%d" % l] = wf.to(op)
            # fp32 copies for the bf16 mode's small-graph SplineConv (_sc_f32)
            d["W%df" % l] = wf
            d["bias%d" % l] = g(pre + ".bias")
        d["aff_w"] = g("vertex_affinity.A.weight")          # [768][1024] = N x K
        d["aff_wT"] = d["aff_w"].t().contiguous()          # [1024][768] for fpm_coef_tanh
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
        # fp64 copies of the AFA-U weights for the fp64 k chain (the GNN packs are read as fp32 and
        # widened in the kernel)
        g64 = lambda k: sd[k].to(device=device, dtype=torch.float64).contiguous()
        f = {}
        for blk in ("row", "col"):
            pre = "encoder_k.layers.0.%s_encoding_block" % blk
            for k, name in (("Wv", ".Wv.weight"), ("mix1w", ".mixed_score_MHA.mix1_weight"),
                            ("mix1b", ".mixed_score_MHA.mix1_bias"), ("mix2w", ".mixed_score_MHA.mix2_weight"),
                            ("mix2b", ".mixed_score_MHA.mix2_bias"), ("Wc", ".multi_head_combine.weight"),
                            ("bc", ".multi_head_combine.bias"), ("W1", ".feed_forward.W1.weight"),
                            ("b1", ".feed_forward.W1.bias"), ("W2", ".feed_forward.W2.weight"),
                            ("b2", ".feed_forward.W2.bias"), ("n1w", ".add_n_normalization_1.norm.weight"),
                            ("n1b", ".add_n_normalization_1.norm.bias"), ("n2w", ".add_n_normalization_2.norm.weight"),
                            ("n2b", ".add_n_normalization_2.norm.bias")):
                f[blk + "_" + k] = g64(pre + name).reshape(-1).contiguous() if k.startswith("mix") else g64(pre + name)
        for h in ("final_row", "final_col"):
            for i in (0, 2):
                f["%s%dw" % (h, i)] = g64("%s.%d.weight" % (h, i)).reshape(-1).contiguous()
                f["%s%db" % (h, i)] = g64("%s.%d.bias" % (h, i))
        d["f64"] = f
        self._pack, self._pack_key = d, key
        self._pack_gen += 1
        return d

    # ------------------------------------------------------------------------------------------
    def plans(self, bt):
        """Spline plans of both sides of ``bt`` (cell masks, product-row tables, dst CSR): shared by
        the two SplineConv layers and the GNN layers of a forward."""
        return [ops.spline_plan(bt.src[s], bt.dst[s], bt.pseudo[s], bt.B * bt.nmax[s], bt.nmax[s],
                                bt.max_graph_edges(s)) for s in range(2)]

    def _spline_side(self, wp, bt, side, cscale, x_op=None, plan=None):
        """SiameseSConvOnNodes over one side's batch (spline_conv.py:28-57) -> operand rows.
        ``x_op``: this side's bf16 operand rows when the caller cast the whole batch up front."""
        dev = bt.device
        f32 = self._sc_f32(bt)
        op = torch.float32 if f32 else torch.bfloat16
        W0, W1 = (wp["W0f"], wp["W1f"]) if f32 else (wp["W0"], wp["W1"])
        nn_ = bt.B * bt.nmax[side]
        E = bt.E[side]
        if plan is None:
            plan = ops.spline_plan(bt.src[side], bt.dst[side], bt.pseudo[side], nn_, bt.nmax[side],
                                   bt.max_graph_edges(side))
        if side == 0 and bt.shared0 and bt.B > 1:
            return (plan,) + self._spline_shared(wp, bt, cscale, probe=x_op if isinstance(x_op, _SharedProbe) else None)
        if isinstance(x_op, _SharedProbe):          # a one-pair chunk of a probe x gallery batch
            x_op = None
        x0 = bt.x[side]
        if x_op is None:
            x_op = ops.cast_bf16(x0) if op == torch.bfloat16 else x0
        yws = ops.spline_y_ws(ops.BF16 if op == torch.bfloat16 else ops.F32, E, nn_, dev)
        h = torch.empty(nn_, C.NODE_FEATURE_DIM, device=dev, dtype=op)
        ops.spline_conv(x_op, plan, E, nn_, bt.nmax[side], bt.n[side], W0, wp["bias0"], yws, 0, out_t=h)
        # bf16 + kp_x3: the vertex affinity's operands as split rows (x2 = A: [hi | lo | hi], x1 o c = B:
        # [hi | hi | lo]) so Kp is a near-fp32 product on the bf16 MFMA path
        split = self._kp_split(side, bt)
        out = torch.empty(nn_, 3 * C.NODE_FEATURE_DIM if split else C.NODE_FEATURE_DIM, device=dev, dtype=op)
        outf = torch.empty(nn_, C.NODE_FEATURE_DIM, device=dev, dtype=torch.float32) if self._keep_feats else None
        ops.spline_conv(h, plan, E, nn_, bt.nmax[side], bt.n[side], W1, wp["bias1"], yws, 1 | (split << 1),
                        xres=x0, cscale=cscale, out_f=outf, out_t=out)
        return plan, out, outf

    def _sc_f32(self, bt):
        """SplineConv products (and the vertex affinity) in fp32 for this batch: the fp32 mode, and the
        bf16 mode on batches whose padded box is at most ``sc_f32_nmax`` keypoints."""
        return self.dtype_mode != "bf16" or max(bt.nmax) <= self.sc_f32_nmax

    def _k_f64(self, bt):
        """The fp64 k chain for this batch (inference forwards on boxes of at most k_f64_nmax keypoints)."""
        return (not self.training) and self.k_f64_nmax > 0 and max(bt.nmax) <= self.k_f64_nmax

    def _kp_split(self, side, bt):
        """Split-operand pattern of side ``side``'s affinity operand rows (0: plain rows)."""
        if self._sc_f32(bt) or not self.kp_x3:
            return 0
        return 2 if side == 0 else 1

    def _spline_shared(self, wp, bt, cscale, probe=None):
        """Probe x gallery: the shared side-0 graph's two SplineConv layers once (pair 0's slice; or
        ``probe``, the forward's prologue result), then broadcast to all pairs with the per-pair
        coefficient scaling (fpm_rows_bcast_scale)."""
        dev = bt.device
        y = probe.y if probe is not None else self._probe_rows(wp, bt)
        nm = bt.nmax[0]
        f32 = self._sc_f32(bt)
        op = torch.float32 if f32 else torch.bfloat16
        split = self._kp_split(0, bt)
        out = torch.empty(bt.B * nm, 3 * C.NODE_FEATURE_DIM if split else C.NODE_FEATURE_DIM, device=dev, dtype=op)
        outf = torch.empty(bt.B * nm, C.NODE_FEATURE_DIM, device=dev, dtype=torch.float32) if self._keep_feats else None
        ops.rows_bcast_scale(y, bt.B, coef=cscale, out_f=outf, out_t=out, split=split)
        return out, outf

    def _probe_rows(self, wp, bt):
        """The shared probe graph's SplineConv output rows (nmax_0, 768) fp32 (both layers, pair 0's
        graph; the same for every chunk of a probe x gallery batch)."""
        dev = bt.device
        f32 = self._sc_f32(bt)
        op = torch.float32 if f32 else torch.bfloat16
        W0, W1 = (wp["W0f"], wp["W1f"]) if f32 else (wp["W0"], wp["W1"])
        nm = bt.nmax[0]
        e0 = int(bt.edge_off[0][1])
        src, dst, ps = bt.src[0][:e0], bt.dst[0][:e0], bt.pseudo[0][:e0]
        plan = ops.spline_plan(src, dst, ps, nm, nm, e0)
        x0 = bt.x[0][:nm]
        nv = bt.n[0][:1]
        x_op = ops.cast_bf16(x0) if op == torch.bfloat16 else x0
        yws = ops.spline_y_ws(ops.BF16 if op == torch.bfloat16 else ops.F32, e0, nm, dev)
        h = torch.empty(nm, C.NODE_FEATURE_DIM, device=dev, dtype=op)
        ops.spline_conv(x_op, plan, e0, nm, nm, nv, W0, wp["bias0"], yws, 0, out_t=h)
        y = torch.empty(nm, C.NODE_FEATURE_DIM, device=dev, dtype=torch.float32)
        ops.spline_conv(h, plan, e0, nm, nm, nv, W1, wp["bias1"], yws, 1, xres=x0, out_f=y)
        return y

    def _afau_norm1_bufs(self, rows, dev):
        """The block's first-norm outputs: fp32 rows and (bf16 modes) the zero-K-padded operand copy."""
        op = torch.bfloat16 if self.afau_mode in ("bf16", "bf16s") else torch.float32
        o1f = torch.empty(rows, C.AFAU_EMB, device=dev, dtype=torch.float32)
        o1t = o1f if op == torch.float32 else torch.empty(rows, C.AFAU_EMB_PAD, device=dev, dtype=op)
        return o1f, o1t

    def _afau_block(self, wp, blk, nb_, P_, mh=None, n2u_d=None, pre=None):
        """One AFA-U encoder block's instance norms + FFN (afau.py:145-199) -> max over positions
        (nb_, E).  "row": on the attention-combine output mh; "col": the synthesised one-hot input
        C0 + combine bias of each distinct n2 (n2u_d).  ``pre``: the first norm's (o1f, o1t) when the
        combine GEMM's epilogue already produced them (fpm_gemm_norm_out)."""
        dev = wp["row_Wc"].device
        op = torch.bfloat16 if self.afau_mode in ("bf16", "bf16s") else torch.float32
        E, FF = C.AFAU_EMB, C.AFAU_FF
        x3 = self.afau_mode == "bf16x3"
        rows = nb_ * P_
        KE = E if op == torch.float32 else C.AFAU_EMB_PAD      # bf16 operand copy: zero-padded K
        o1f, o1t = pre if pre is not None else self._afau_norm1_bufs(rows, dev)
        if pre is None and blk == "row":
            ops.instnorm(mh, nb_, P_, E, wp["row_n1w"], wp["row_n1b"], out_f=o1f,
                         out_t=None if op == torch.float32 else o1t, ldt=KE)
        elif pre is None:
            ops.instnorm(None, nb_, P_, E, wp["col_n1w"], wp["col_n1b"], nvalid=n2u_d, onehot_bias=wp["col_bc"],
                         out_f=o1f, out_t=None if op == torch.float32 else o1t, ldt=KE)
        ff = torch.empty(rows, E, device=dev, dtype=torch.float32)
        if x3:
            # o1t: the split [hi | lo | hi] copy when the combine GEMM's epilogue wrote it
            o13 = o1t if o1t is not o1f else ops.split_bf16x3(o1f, C.AFAU_EMB_PAD)
            if P_ in (128, 256) and self.afau_fuse_norm:
                # W1 + bias + ReLU straight into split operands, then W2 with the block tail (instance
                # norm + max over the pair's 256 positions) in its epilogue: no fp32 FFN round trip
                h3 = ops.gemm_x3out(o13, wp[blk + "_W1"], rows, FF, 3 * C.AFAU_EMB_PAD, FF, epi=ops.EPI_RELU,
                                    bias=wp[blk + "_b1"])
                gm = torch.empty(nb_, E, device=dev, dtype=torch.float32)
                return ops.gemm_norm_max(h3, wp[blk + "_W2"], rows, E, 3 * FF, 3 * FF, 3 * FF, wp[blk + "_b2"], o1f,
                                         wp[blk + "_n2w"], wp[blk + "_n2b"], gm, P=P_)
            hf = torch.empty(rows, FF, device=dev, dtype=torch.float32)
            ops.gemm(o13, wp[blk + "_W1"], rows, FF, 3 * C.AFAU_EMB_PAD, o13.shape[1], o13.shape[1],
                     epi=ops.EPI_RELU, bias=wp[blk + "_b1"], out_f=hf, ldc=FF)
            h3 = ops.split_bf16x3(hf, FF)
            ops.gemm(h3, wp[blk + "_W2"], rows, E, 3 * FF, h3.shape[1], h3.shape[1], bias=wp[blk + "_b2"],
                     out_f=ff, ldc=E)
        else:
            hbuf = torch.empty(rows, FF, device=dev, dtype=op)
            ops.gemm(o1t, wp[blk + "_W1"], rows, FF, KE, KE, KE, epi=ops.EPI_RELU, bias=wp[blk + "_b1"],
                     out_t=hbuf if op != torch.float32 else None, out_f=hbuf if op == torch.float32 else None,
                     ldc=FF)
            if op != torch.float32 and P_ in (128, 256) and self.afau_fuse_norm:
                # the second GEMM's epilogue takes the instance norm + max over the pair's 256
                # positions (one GEMM tile): the (rows x 600) FFN output never reaches HBM
                gm = torch.empty(nb_, E, device=dev, dtype=torch.float32)
                return ops.gemm_norm_max(hbuf, wp[blk + "_W2"], rows, E, FF, FF, FF, wp[blk + "_b2"], o1f,
                                         wp[blk + "_n2w"], wp[blk + "_n2b"], gm, P=P_)
            ops.gemm(hbuf, wp[blk + "_W2"], rows, E, FF, FF, FF, bias=wp[blk + "_b2"], out_f=ff, ldc=E)
        gm = torch.empty(nb_, E, device=dev, dtype=torch.float32)
        ops.instnorm(o1f, nb_, P_, E, wp[blk + "_n2w"], wp[blk + "_n2b"], in2=ff, gmax=gm)
        return gm

    @staticmethod
    def _afau_col_index(bt):
        """(distinct n2 values, their device copy, per-pair gather index or None) of a batch; cached on
        the batch object (its sizes do not change), so a repeated forward makes no host work or
        host-to-device copy here."""
        cached = getattr(bt, "_afau_col_idx", None)
        if cached is not None and cached[1].device == bt.device:
            return cached
        n2u = np.unique(bt.n_host[1].numpy())
        n2u_d = torch.as_tensor(n2u, dtype=torch.int32).to(bt.device, non_blocking=True)
        n2c = bt.n_host[1].numpy()
        inv = None
        if len(n2u) != len(n2c) or not np.array_equal(n2u, n2c):
            inv = torch.as_tensor(np.searchsorted(n2u, n2c), dtype=torch.long).to(bt.device, non_blocking=True)
        try:
            bt._afau_col_idx = (n2u, n2u_d, inv)
        except AttributeError:
            pass
        return n2u, n2u_d, inv

    def _afau_col(self, wp, bt, idx=None):
        """The AFA-U column block for every distinct n2 of a batch: (n2u, gmax per n2u, n2max, gather
        index or None).  The column block sees a = one-hot rows and b = zero rows, so k = v = 0 and
        its attention output is exactly the combine bias (afau.py:99-142): its result depends on n2
        and the batch's n2max only, not on ss.  A forward computes it once per distinct n2 and
        gathers it for every pair and pipeline chunk -- the same arithmetic on the same inputs,
        bit-identical to the per-pair evaluation.  The host-to-device index copies happen here, once
        per batch (``idx`` = _afau_col_index(bt), computed before a graph capture)."""
        n2u, n2u_d, inv = idx if idx is not None else self._afau_col_index(bt)
        return n2u, self._afau_block(wp, "col", len(n2u), bt.n2max, n2u_d=n2u_d), bt.n2max, inv

    def _afau(self, wp, ss, bt, col=None, b0=0):
        """AFA-U k regression (ngm.py:386-412) -> ks (B,).  ``col``: the _afau_col result of the
        forward's batch, whose pairs [b0, b0 + B) this (sub-)batch is (computed here when None)."""
        dev = ss.device
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        # f32 / bf16x3: fp32 activations; bf16 / bf16s: bf16 FFN operands
        op = torch.bfloat16 if self.afau_mode in ("bf16", "bf16s") else torch.float32
        E, HD = C.AFAU_EMB, C.AFAU_HEADS * C.AFAU_QKV
        if max(n1max, n2max) > self.univ_size:
            raise AssertionError("UNIV_SIZE cap: n1max/n2max must be <= %d (ngm.py:387-389)" % self.univ_size)
        x3 = self.afau_mode == "bf16x3"          # near-fp32 products on bf16 MFMA (split operands)
        # bf16s / bf16x3: the attention kernel writes its output as split rows [hi | lo | hi]
        split = self.afau_mode in ("bf16s", "bf16x3")
        att = torch.empty(B * n1max, 3 * HD if split else HD, device=dev,
                          dtype=torch.bfloat16 if split else op)
        ops.crossset_attn(ss, bt.n2, wp["row_Wv"], wp["row_mix1w"], wp["row_mix1b"], wp["row_mix2w"],
                          wp["row_mix2b"], att, split=split)
        # bf16s: hi*W_hi + lo*W_hi (2 terms); bf16x3: + hi*W_lo (3 terms, near-fp32)
        kc = 3 * HD if x3 else (2 * HD if split else HD)
        # fused instance norms: a pair's positions are one 256-row GEMM tile or half of one (128)
        fuse = self.afau_fuse_norm and n1max in (128, 256)
        if x3 and fuse:
            # the combine projection + first instance norm in one GEMM, its output both as fp32 rows
            # (the block's residual) and as the split operand of the FFN's first product
            o1f = torch.empty(B * n1max, E, device=dev, dtype=torch.float32)
            o13 = ops.gemm_x3out(att, wp["row_Wc"], B * n1max, E, kc, C.AFAU_EMB_PAD, epi=ops.EPI_NORM_OUT,
                                 bias=wp["row_bc"], out_f=o1f, nw=wp["row_n1w"], nb=wp["row_n1b"], P=n1max)
            g_row = self._afau_block(wp, "row", B, n1max, pre=(o1f, o13))
        elif att.dtype == torch.bfloat16 and not x3 and fuse:
            # the combine projection's epilogue applies the block's first instance norm (one GEMM
            # tile = one pair's 256 positions): mh never reaches HBM un-normalised
            o1f, o1t = self._afau_norm1_bufs(B * n1max, dev)
            ops.gemm_norm_out(att, wp["row_Wc"], B * n1max, E, kc, att.shape[1], att.shape[1], wp["row_bc"],
                              wp["row_n1w"], wp["row_n1b"], o1f, out_t=None if o1t is o1f else o1t, P=n1max)
            g_row = self._afau_block(wp, "row", B, n1max, pre=(o1f, o1t))
        else:
            mh = torch.empty(B * n1max, E, device=dev, dtype=torch.float32)
            ops.gemm(att, wp["row_Wc"], B * n1max, E, kc, att.shape[1], att.shape[1], bias=wp["row_bc"], out_f=mh,
                     ldc=E)
            g_row = self._afau_block(wp, "row", B, n1max, mh=mh)
        if col is None or isinstance(col[0], str) or col[2] != n2max:
            col, b0 = self._afau_col(wp, bt), 0
        n2u, gm_u, _, inv = col
        g_col = gm_u if inv is None else gm_u.index_select(0, inv[b0:b0 + B])
        ks = torch.empty(B, device=dev, dtype=torch.float32)
        ops.afau_head(g_row, g_col, B, E, wp["final_row0w"], wp["final_row0b"], wp["final_row2w"],
                      wp["final_row2b"], wp["final_col0w"], wp["final_col0b"], wp["final_col2w"], wp["final_col2b"], ks)
        return ks

    def _afau_col_f64(self, wp, bt, idx=None):
        """The AFA-U column block in fp64 (independent of ss: one-hot rows + the combine bias) once per
        distinct n2 of the batch -> ("f64", pooled rows (U, E) fp64, n2max, int32 gather index or
        None); ``idx`` = _afau_col_index(bt) (computed before any graph capture)."""
        f = wp["f64"]
        n2u, n2u_d, inv = idx if idx is not None else self._afau_col_index(bt)
        U, n2max, E = len(n2u), bt.n2max, C.AFAU_EMB
        f64 = dict(device=bt.device, dtype=torch.float64)
        o1c = torch.empty(U * n2max, E, **f64)
        ops.instnorm_f64(None, U, n2max, E, f["col_n1w"], f["col_n1b"], nvalid=n2u_d, onehot_bias=f["col_bc"], out=o1c)
        ffc = ops.gemm_f64(ops.gemm_f64(o1c, f["col_W1"], f["col_b1"], relu=True), f["col_W2"], f["col_b2"])
        g_col = torch.empty(U, E, **f64)
        ops.instnorm_f64(o1c, U, n2max, E, f["col_n2w"], f["col_n2b"], in2=ffc, gmax=g_col)
        return "f64", g_col, n2max, None if inv is None else inv.to(torch.int32)

    def _afau_f64(self, wp, ss64, bt, col=None, b0=0):
        """AFA-U k regression (ngm.py:386-412) in fp64 from the fp64 ss (the fp64 k chain) -> ks (B,)
        fp32.  Row block: attention, combine, norm, FFN, norm + max-pool; col block: ``col`` =
        _afau_col_f64 of the forward's batch, whose pairs [b0, b0 + B) this (sub-)batch is (computed
        here when None)."""
        f = wp["f64"]
        dev = ss64.device
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        E, HD = C.AFAU_EMB, C.AFAU_HEADS * C.AFAU_QKV
        if max(n1max, n2max) > self.univ_size:
            raise AssertionError("UNIV_SIZE cap: n1max/n2max must be <= %d (ngm.py:387-389)" % self.univ_size)
        f64 = dict(device=dev, dtype=torch.float64)
        att = torch.empty(B * n1max, HD, **f64)
        ops.crossset_attn_row_f64(ss64, bt.n2, f["row_Wv"], f["row_mix1w"], f["row_mix1b"], f["row_mix2w"],
                                  f["row_mix2b"], att)
        mh = ops.gemm_f64(att, f["row_Wc"], f["row_bc"])
        o1 = torch.empty_like(mh)
        ops.instnorm_f64(mh, B, n1max, E, f["row_n1w"], f["row_n1b"], out=o1)
        ff = ops.gemm_f64(ops.gemm_f64(o1, f["row_W1"], f["row_b1"], relu=True), f["row_W2"], f["row_b2"])
        g_row = torch.empty(B, E, **f64)
        ops.instnorm_f64(o1, B, n1max, E, f["row_n2w"], f["row_n2b"], in2=ff, gmax=g_row)
        if col is None or not isinstance(col[0], str) or col[2] != n2max:
            col, b0 = self._afau_col_f64(wp, bt), 0
        _, g_col, _, inv = col
        ks = torch.empty(B, device=dev, dtype=torch.float32)
        ops.afau_head_f64(g_row, g_col, None if inv is None else inv[b0:b0 + B], B, E, f["final_row0w"],
                          f["final_row0b"], f["final_row2w"], f["final_row2b"], f["final_col0w"], f["final_col0b"],
                          f["final_col2w"], f["final_col2b"], ks)
        return ks

    def _gnn_chain_f64(self, wp, bt, Kp, csr1, csr2, s, ss, ss64):
        """The three GNN layers (+ their Sinkhorns), the readout and the final Sinkhorn in fp64
        (csrc/precise.hip) from the fp32 Kp: writes s / ss (fp32 copies) and ss64."""
        dev = bt.device
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        f64 = dict(device=dev, dtype=torch.float64)
        X, Cin = Kp, 1
        zbuf = torch.empty(B, n2max, n1max, **f64)
        for l in range(C.GNN_LAYER):
            Xn = torch.empty(B, 17, n2max, n1max, **f64)
            ops.gnn_layer_f64(X, Cin, B, n1max, n2max, csr1, csr2, bt.n1, bt.n2, wp["gnn%d" % l], Xn, zbuf)
            ops.sinkhorn_f64(zbuf.transpose(1, 2), bt.n1, bt.n2, C.GNN_SK_ITER, self.tau, True,
                             out=Xn[:, 16].transpose(1, 2))
            X, Cin = Xn, 17
            self._mark("gnn%d" % l)
        s64 = torch.empty(B, n1max, n2max, **f64)
        ops.node_classifier_f64(X, B, n1max, n2max, wp["cls_w"], wp["cls_b"], s64, s)
        ops.sinkhorn_f64(s64, bt.n1, bt.n2, C.SK_ITER_NUM, self.tau, True, out=ss64, out32=ss)

    def _mark(self, name):
        """Diagnostic stage timing (FPM_STAGE_TIMING=1): synchronises, so never in timed runs.
        FPM_STAGE_EVENTS=1: a timing event on the current stream per mark instead (no sync; for
        one-stream forwards, stage_events() gives the GPU time between consecutive marks)."""
        if self._stage_events:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream())
            self._ev_marks.append((name, ev))
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
        ops.coef_tanh(gw, wp["aff_wT"], wp["aff_b"], coef)
        return gw, coef

    def run_gpu_stage(self, bt, keep_feats=False, s_out=None, ss_out=None, gc=None, x_ops=(None, None), plans=None,
                      ss64_out=None):
        """Everything up to ss on the GPU.  Returns a dict of device tensors.  ``gc``: this
        batch's rows of global_coef() when computed for a parent batch; ``x_ops``: its rows of the
        parent's bf16 operand copies of the node features (cast once per forward); ``plans``:
        plans(bt) when already computed; ``ss64_out``: the fp64 ss of the fp64 k chain (_k_f64)."""
        keep_feats = keep_feats or self.compute_ke
        self._keep_feats = keep_feats
        if self._stage_timing:
            torch.cuda.synchronize()
            self._t_last = time.perf_counter()
        self._mark("start")
        wp = self.packed(bt.device)
        dev = bt.device
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        N = n1max * n2max
        gw, coef = gc if gc is not None else self.global_coef(bt)
        self._mark("coef")
        pl = plans if plans is not None else self.plans(bt)
        plan0, x1c, f1 = self._spline_side(wp, bt, 0, coef, x_ops[0], pl[0])
        self._mark("splineconv0")
        plan1, x2, f2 = self._spline_side(wp, bt, 1, None, x_ops[1], pl[1])
        self._mark("splineconv")
        # Kp^T per pair: emb0[b][j][i] = softplus((x1_i o c) . x2_j) - 0.5 on the valid block (ngm.py:277-321)
        X = torch.empty(B, 1, n2max, n1max, device=dev, dtype=torch.float32)
        # split operand rows (bf16 + kp_x3): K = 3 x 768, hi.hi + lo.hi + hi.lo (near-fp32 Kp)
        Kk = x2.shape[1]
        ops.gemm(x2, x1c, n2max, n1max, Kk, Kk, Kk, batch=B, sA=n2max * Kk, sB=n1max * Kk, epi=ops.EPI_AFFINITY,
                 out_f=X, ldc=n1max, sC=N, n1=bt.n1, n2=bt.n2)
        Kp = X
        Ke = self._edge_affinity(wp, bt, gw, f1, f2) if self.compute_ke else None
        self._mark("affinity")
        csr1 = ops.plan_csr(plan0, bt.E[0], B * n1max)
        csr2 = ops.plan_csr(plan1, bt.E[1], B * n2max)
        if self._k_f64(bt):
            s = s_out if s_out is not None else torch.empty(B, n1max, n2max, device=dev, dtype=torch.float32)
            ss = ss_out if ss_out is not None else torch.empty(B, n1max, n2max, device=dev, dtype=torch.float32)
            ss64 = ss64_out if ss64_out is not None else torch.empty(B, n1max, n2max, device=dev, dtype=torch.float64)
            self._gnn_chain_f64(wp, bt, Kp, csr1, csr2, s, ss, ss64)
            self._mark("final_sinkhorn")
            out = dict(s=s, ss=ss, ss64=ss64, Kp=Kp[:, 0].transpose(1, 2), coef=coef)
            if keep_feats:
                out["feat0"], out["feat1"] = f1, f2
            if Ke is not None:
                out["Ke"] = Ke
            return out
        zbuf = torch.empty(B, n2max, n1max, device=dev, dtype=torch.float32)
        vpart = torch.empty(B, n2max, n1max, device=dev, dtype=torch.float32)
        Cin = 1
        for l in range(C.GNN_LAYER):
            Xn = torch.empty(B, 17, n2max, n1max, device=dev, dtype=torch.float32)
            last = l == C.GNN_LAYER - 1      # fuse the final classifier's x1 part (ngm.py:368)
            ops.gnn_layer(X, Cin, B, n1max, n2max, csr1, csr2, bt.n1, bt.n2, wp["gnn%d" % l], Xn, zbuf,
                          vpart=vpart if last else None, cls_w=wp["cls_w"] if last else None,
                          ord2=getattr(bt, "ord2", None))
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
            self._stream_cache[key] = [torch.cuda.Stream(dev) for _ in range(self.n_streams)]
        return self._stream_cache[key]

    def _lsa_streams(self, dev):
        key = "lsa:" + str(dev)
        if key not in self._stream_cache:
            self._stream_cache[key] = [torch.cuda.Stream(dev) for _ in range(2)]
        return self._stream_cache[key]

    def _tail_extra_streams(self, dev):
        key = "tail:" + str(dev)
        if key not in self._stream_cache:
            self._stream_cache[key] = [torch.cuda.Stream(dev) for _ in range(2)]
        return self._stream_cache[key]

    def _copy_stream(self, dev):
        key = "copy:" + str(dev)
        if key not in self._stream_cache:
            self._stream_cache[key] = torch.cuda.Stream(dev)
        return self._stream_cache[key]

    def pipeline_chunks(self, B):
        """Sub-batches per forward so the host Hungarian of chunk c overlaps the GPU work of c+1."""
        if self.chunks is not None:
            return max(1, min(self.chunks, B))
        if os.environ.get("FPM_CHUNKS"):
            return max(1, min(int(os.environ["FPM_CHUNKS"]), B))
        # FPM_CHUNK_MIN: fewest pairs per chunk (A/B for small per-GPU batches)
        return max(1, min(8, B // int(os.environ.get("FPM_CHUNK_MIN", "128"))))

    def _enqueue_copy(self, dev, b0, b1, o, done, after=None):
        """ds_mat[b0:b1] -> pinned host memory on the copy stream (the copy is a blit kernel: on a
        stream of its own it does not hold back the next chunk queued on a compute stream) once
        ``done`` (and ``after``, if given) have fired; returns the copy's completion event, which
        the host thread waits on with a sleeping (not spinning) wait, leaving its core to the
        Hungarian pool."""
        cs = self._copy_stream(dev)
        cs.wait_event(done)
        if after is not None:
            cs.wait_event(after)
        with torch.cuda.stream(cs):
            self._pinned[b0:b1].copy_(o["ds_mat"][b0:b1], non_blocking=True)
        ev = torch.cuda.Event(enable_timing=True, blocking=True)
        ev.record(cs)
        return ev

    def _stage_a(self, part, b0, b1, o, keep_feats, gt_ks, min_pt, gc, col=None, xop=None, plans=None,
                 tail=None, zc=False):
        """GPU stage of one chunk (on the current stream): everything up to ds_mat.  Only device
        work on tensors that outlive the call (capturable into a HIP graph).  ``tail``: a callback
        that splits the chunk's tail (AFA-U, soft top-k) into pair sub-ranges -- called with
        (tail view, b0, b1) right after each sub-range's soft top-k is queued."""
        dev = part.device
        x_ops = tuple(None if t is None else t if isinstance(t, _SharedProbe) else t[b0 * part.nmax[s]:b1 * part.nmax[s]]
                      for s, t in enumerate(xop or (None, None)))
        r = self.run_gpu_stage(part, keep_feats, s_out=o["s"][b0:b1], ss_out=o["ss"][b0:b1],
                               gc=(gc[0][b0:b1], gc[1][b0:b1]), x_ops=x_ops, plans=plans,
                               ss64_out=o["ss64"][b0:b1] if "ss64" in o else None)
        if tail is None:
            self._stage_tail(part, b0, b1, o, gt_ks, min_pt, col, host=self._pinned[b0:b1] if zc else None)
            return r
        cur = torch.cuda.current_stream(dev)
        ranges = self._tail_ranges(b0, b1)
        rot = [cur]
        if self.tail_streams > 1 and len(ranges) > 1 and self.n_streams > 1:
            alt = next((st for st in self._streams(dev) if st != cur), None)
            if alt is not None:
                rot.append(alt)
                rot += self._tail_extra_streams(dev)[:self.tail_streams - 2]
        if len(rot) > 1:
            ev_ss = torch.cuda.Event()
            ev_ss.record(cur)
            for st in rot[1:]:
                st.wait_event(ev_ss)
        for k, (sb0, sb1) in enumerate(ranges):
            view = _TailView(part, sb0 - b0, sb1 - b0, (sb0, sb1))
            with torch.cuda.stream(rot[k % len(rot)]):
                self._stage_tail(view, sb0, sb1, o, gt_ks, min_pt, col,
                                 host=self._pinned[sb0:sb1] if zc else None)
                tail(view, sb0, sb1)
        for st in rot[1:]:
            cur.wait_stream(st)        # the forward's later work on cur sees every group's outputs
        return r

    def _stage_tail(self, part, b0, b1, o, gt_ks, min_pt, col, host=None):
        """AFA-U k regression + soft top-k of pairs [b0, b1) (``part`` covers exactly them).  ``host``:
        the pinned rows of the host Hungarian, written by the soft top-k kernel itself (zero-copy)."""
        dev = part.device
        ks = o["k_prob"][b0:b1]
        if self.regression and "ss64" in o:
            ks.copy_(self._afau_f64(self.packed(dev), o["ss64"][b0:b1], part, col=col, b0=b0))
        elif self.regression:
            ks.copy_(self._afau(self.packed(dev), o["ss"][b0:b1], part, col=col, b0=b0))
        else:
            ks.copy_(gt_ks[b0:b1] / min_pt[b0:b1])
        self._mark("afau")
        k_used = gt_ks[b0:b1] if self.training else ks * min_pt[b0:b1]
        if "ss64" in o:
            # the fp64 k chain carries on through the soft top-k (its tau = 0.01 2-column Sinkhorn
            # amplifies ss's fp32 rounding on small boxes as the final Sinkhorn does)
            ops.soft_topk_f64(o["ss64"][b0:b1], part.n1, part.n2, k_used.contiguous(), C.SK_ITER_NUM, self.tau,
                              out=o["ds_mat"][b0:b1], steps=o["sk_steps"][b0:b1], out_host=host)
        else:
            ops.soft_topk_fwd(o["ss"][b0:b1], part.n1, part.n2, k_used.contiguous(), C.SK_ITER_NUM, self.tau,
                              out=o["ds_mat"][b0:b1], steps=o["sk_steps"][b0:b1], out_host=host)
        o["_kk"][b0:b1].copy_(ks * min_pt[b0:b1])
        self._mark("soft_topk")

    def _tail_ranges(self, b0, b1):
        """Sub-ranges of a one-chunk forward's tail (FPM_TAIL_GROUPS, default 4): equal groups, the last
        one ``tail_last`` (FPM_TAIL_LAST, default 0.5) of the others' size -- its Hungarian is the part
        of the host work no later GPU work hides, while every group costs about the same GPU latency."""
        g = max(1, min(self.tail_groups, (b1 - b0) // max(1, self.tail_min)))
        w = [1.0] * (g - 1) + [self.tail_last if g > 1 else 1.0]
        tot = sum(w)
        acc, bounds = 0.0, [b0]
        for x in w[:-1]:
            acc += x
            bounds.append(b0 + round(acc * (b1 - b0) / tot))
        bounds.append(b1)
        return [(bounds[i], bounds[i + 1]) for i in range(g) if bounds[i + 1] > bounds[i]]

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

    def _stage_c(self, part, b0, b1, o, assign=None):
        """Host Hungarian (utils/hungarian.py: LSA of -ds_mat per pair) + greedy selection +
        MatchClassifier of one chunk; the caller waits for the chunk's D2H event first.  ``assign``:
        the chunk's assignment when its Hungarian already ran (ops.lsa_submit)."""
        dev = part.device
        wp = self._pack
        t = time.perf_counter()
        if assign is None:
            assign = ops.lsa_batch_host(self._pinned[b0:b1], part.n_host[0], part.n_host[1], self.lsa_threads, b0=b0,
                                        out=self._assign_pinned[b0:b1])
        dt = time.perf_counter() - t
        assign_d = assign.to(dev, non_blocking=True)      # pinned (self._assign_pinned): asynchronous
        ops.topk_select(o["ds_mat"][b0:b1], assign_d, o["_kk"][b0:b1], lsa_out=o["lsa"][b0:b1],
                        out=o["perm_mat"][b0:b1])
        self._mark("lsa+h2d+select")
        ops.match_cls(o["s"][b0:b1], o["perm_mat"][b0:b1], wp["mc_w1"], wp["mc_b1"], wp["mc_sc1"], wp["mc_sh1"],
                      wp["mc_w2"], wp["mc_b2"], wp["mc_sc2"], wp["mc_sh2"], wp["mc_fcw"], wp["mc_fcb"],
                      logits=o["cls_logits"][b0:b1], prob=o["cls_prob"][b0:b1],
                      dtype=ops.BF16 if self.dtype_mode == "bf16" else ops.F32)
        self._mark("match_cls")
        return dt

    @staticmethod
    def _alloc_outputs(B, n1max, n2max, dev, k_f64=False):
        f32 = dict(device=dev, dtype=torch.float32)
        o = {k: torch.empty(B, n1max, n2max, **f32) for k in ("s", "ss", "ds_mat", "perm_mat", "lsa")}
        if k_f64:
            o["ss64"] = torch.empty(B, n1max, n2max, device=dev, dtype=torch.float64)
        o.update({k: torch.empty(B, **f32) for k in ("k_prob", "cls_logits", "cls_prob", "_kk")})
        o["sk_steps"] = torch.empty(B, device=dev, dtype=torch.int32)
        o["_lsa_status"] = torch.zeros(B, device=dev, dtype=torch.int32)
        return o

    def _prologue(self, bt, parts, cast=True, col_idx=None, fork=True, plans_one=False):
        """Per-forward work before the chunks (main stream): global weights + affinity
        coefficients, the bf16 operand rows of both sides' node features in one launch each (before
        any chunk's ds_mat D2H is in flight: cast per chunk, they ran beside the copy's blit kernel
        and stalled ~14x; a shared probe side is cast inside its chunk's one-graph SplineConv), the
        AFA-U column block once per distinct n2, and every chunk's spline plans (one launch per plan
        kernel and side for all chunks, ops.spline_plans_multi: dozens of small latency-bound
        launches, which stalled ~10x when they ran beside a ds_mat D2H blit, become six, before any
        copy is in flight) -> (gc, xop, col, plans per chunk or None).
        ``fork`` (eager forwards): the HBM-bound casts and the AFA-U column block run on a side stream
        beside the latency-bound plan kernels and coefficients, joined before the chunks start."""
        dev = bt.device
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev) if (fork and self.prologue_fork) else None
        if side is not None:
            ev_fork = torch.cuda.Event()
            ev_fork.record(main)
            side.wait_event(ev_fork)

        def side_work():
            xop_ = None
            if not self._sc_f32(bt) and cast:
                xop_ = tuple(None if (s == 0 and bt.shared0) else ops.cast_bf16(bt.x[s]) for s in range(2))
                if bt.shared0 and bt.B > 1:
                    # the probe's SplineConv once per forward, not once per chunk
                    xop_ = (_SharedProbe(self._probe_rows(self.packed(dev), bt)), xop_[1])
            self._mark("pro_cast")
            col_ = None
            if self.regression:
                col_ = (self._afau_col_f64 if self._k_f64(bt) else self._afau_col)(self.packed(dev), bt, col_idx)
            return xop_, col_
        if side is not None:
            with torch.cuda.stream(side):
                xop, col = side_work()
            ev_join = torch.cuda.Event()
            ev_join.record(side)
        pre = None
        if len(parts) > 1 or plans_one:
            pre = [ops.spline_plans_multi(parts, s, bt.nmax[s]) for s in range(2)]
            pre = None if any(p is None for p in pre) else [list(pc) for pc in zip(*pre)]
        self._mark("pro_plans")
        gc = self.global_coef(bt)
        self._mark("pro_coef")
        if side is None:
            xop, col = side_work()
        else:
            main.wait_event(ev_join)
        self._mark("prologue")
        return gc, xop, col, pre

    def _side_stream(self, dev):
        # the copy stream: idle until the first chunk's D2H, and no extra stream (hardware queues are
        # few: GPU_MAX_HW_QUEUES = 4 -- more streams than queues share them)
        return self._copy_stream(dev)

    def _graph_state(self, bt, parts, dev):
        """HIP graphs of one batch's forward, captured on first use and replayed while the batch,
        the chunking and the packed weights stay the same: the prologue on the main stream, then per
        chunk its spline plans and the rest of its GPU stage (two graphs, so the copy deferral can
        wait between them) on the chunk's stream.  Chunks of one stream share a memory pool (they
        run in order); the two streams and the prologue have their own.  Every tensor a graph reads
        or writes outside its pool is a static buffer of the state."""
        wp = self.packed(dev)
        rng = [(0, bt.B) if p is bt else p.pair_range for p in parts]
        # everything a captured launch bakes in: sizes, modes, packed weights, tau (a kernel argument),
        # the fused-norm switch and the kernel-variant switches (ops.set_tuning)
        key = (len(parts), tuple(rng), self.dtype_mode, self.afau_mode, self.kp_x3, self.regression,
               self.n_streams, self._pack_gen, str(dev), float(self.tau), self.afau_fuse_norm,
               ops.tuning_generation(), self.sc_f32_nmax, self.k_f64_nmax)
        g = self._gstate
        if g is not None and g["bt"]() is bt and g["key"] == key:
            return g
        self._gstate = None
        torch.cuda.synchronize(dev)
        import weakref
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        g = {"bt": weakref.ref(bt), "key": key}
        o = self._alloc_outputs(B, n1max, n2max, dev, k_f64=self._k_f64(bt))
        g["o"] = o
        g["min_pt"] = torch.minimum(bt.n1, bt.n2).to(torch.float32)
        g["gt_ks"] = g["min_pt"].clone()
        streams = self._streams(dev)
        pools = [torch.cuda.graph_pool_handle() for _ in range(len(streams) + 1)]
        g["col_idx"] = self._afau_col_index(bt) if self.regression else None
        if len(parts) > 1:                    # the multi-plan job tables (host-to-device copies)
            for s_ in range(2):
                ops.spline_plan_jobs(parts, s_, bt.nmax[s_])
        torch.cuda.synchronize(dev)
        gp = torch.cuda.CUDAGraph()
        # captured on a side stream (capture needs a non-default stream), replayed on the main one
        with torch.cuda.graph(gp, pool=pools[-1], stream=self._copy_stream(dev)):
            gc, xop, col, pre = self._prologue(bt, parts, col_idx=g["col_idx"], fork=False)
        g["prologue"], g["pro_out"] = gp, (gc, xop, col, pre)
        g["chunks"] = []
        for c, part in enumerate(parts):
            st = streams[c % len(streams)]
            b0, b1 = rng[c]
            gpl, gst = None, torch.cuda.CUDAGraph()
            if pre is not None:
                pl = pre[c]
            else:
                gpl = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gpl, pool=pools[c % len(streams)], stream=st):
                    pl = self.plans(part)
            with torch.cuda.graph(gst, pool=pools[c % len(streams)], stream=st):
                self._stage_a(part, b0, b1, o, False, g["gt_ks"], g["min_pt"], gc, col=col, xop=xop, plans=pl)
            g["chunks"].append((gpl, gst, pl))
        torch.cuda.synchronize(dev)
        self._gstate = g
        return g

    def _prologue_replay(self, bt, parts, dev):
        """The eager forward's prologue from a HIP graph (FPM_PROLOGUE_GRAPH): captured once per
        (batch, chunking, packed weights, modes) on the copy stream, replayed on the main stream
        (which orders it after the previous forward); its outputs live in the graph's pool and are
        rewritten by each replay.  None when the forward must run the prologue eagerly."""
        if (not self.prologue_graph or (self.prologue_graph == 1 and len(parts) > 1)
                or self.training or self._stage_timing or self._stage_events
                or ops.profiling() or self._enqueue_lock is not None):
            return None
        self.packed(dev)                      # (re)packed weights outside any capture; sets _pack_gen
        rng = tuple((0, bt.B) if p is bt else p.pair_range for p in parts)
        key = (len(parts), rng, self.dtype_mode, self.afau_mode, self.kp_x3, self.regression, self._pack_gen,
               str(dev), self.afau_fuse_norm, ops.tuning_generation(), self.sc_f32_nmax, self.k_f64_nmax)
        g = self._pgstate
        if g is None or g["bt"]() is not bt or g["key"] != key:
            import weakref
            self._pgstate = None
            torch.cuda.synchronize(dev)
            col_idx = self._afau_col_index(bt) if self.regression else None
            for s_ in range(2):               # the multi-plan job tables (host-to-device copies)
                ops.spline_plan_jobs(parts, s_, bt.nmax[s_])
            torch.cuda.synchronize(dev)
            gp = torch.cuda.CUDAGraph()
            # one-chunk forwards too: their casts and spline plans join the replayed prologue
            with torch.cuda.graph(gp, stream=self._copy_stream(dev)):
                out = self._prologue(bt, parts, cast=True, col_idx=col_idx, fork=False, plans_one=True)
            g = self._pgstate = {"bt": weakref.ref(bt), "key": key, "graph": gp, "out": out}
        g["graph"].replay()
        return g["out"]

    def _parts(self, bt, chunks=None):
        K = chunks if chunks is not None else self.pipeline_chunks(bt.B)
        if self.compute_ke:
            K = 1          # Ke blocks are padded to per-chunk edge maxima: keep one chunk
        return bt.split(K, self.tail_splits if K > 1 else 0)

    def _graphed(self, parts, keep_feats=False):
        return (self.use_graphs and not keep_feats and self.lsa_mode != "device" and not self.compute_ke
                and not self.training and not self._stage_timing and not self._stage_events and not ops.profiling())

    def stage_events(self, reset=True, absolute=False):
        """FPM_STAGE_EVENTS=1: [(stage, ms since the previous mark)] of the marks recorded so far
        (synchronises); meaningful for one-stream forwards.  ``absolute``: [(stage, ms since the first
        mark)] sorted by time -- the GPU timeline of stage completions over all streams."""
        torch.cuda.synchronize()
        out, prev = [], None
        first = self._ev_marks[0][1] if self._ev_marks else None
        for name, ev in self._ev_marks:
            if absolute:
                out.append((name, first.elapsed_time(ev)))
            elif prev is not None:
                out.append((name, prev.elapsed_time(ev)))
            prev = ev
        if reset:
            self._ev_marks = []
        return sorted(out, key=lambda t: t[1]) if absolute else out

    def prepare(self, bt, chunks=None):
        """Capture ``bt``'s HIP graphs now if its forward will replay them (graph mode, multi-chunk),
        so the first run() only replays -- e.g. before several host threads drive their devices."""
        parts = self._parts(bt, chunks)
        if self._graphed(parts):
            with torch.cuda.device(bt.device):
                self._graph_state(bt, parts, bt.device)

    def run(self, bt, gt_perm=None, label=None, keep_feats=False, chunks=None):
        """Full forward, pipelined over sub-batches ("chunks").  Every chunk's GPU stage is queued
        at once, alternating over two streams (per-pair kernels of neighbouring chunks -- Sinkhorn,
        soft top-k, AFA-U, one workgroup per pair -- then fill the 256 CUs together); the host LSA
        of chunk c starts as soon as its ds_mat lands in pinned memory while the GPU continues;
        chunk c's selection + classifier follow its LSA on its stream.

        With ``use_graphs`` (FPM_GRAPHS=1, ShardedNet's replicas), inference forwards replay HIP
        graphs of the prologue and of every chunk's GPU stage (captured on the batch's first
        forward, _graph_state): ~100 kernel launches per chunk become two graph launches.  Graph
        mode returns fresh copies of the
        reference outputs (ds_mat, perm_mat, k_prob, cls_prob); s / ss / lsa are views of the
        batch's static buffers, valid until its next forward."""
        if ops.timing_probes_on():
            raise ops._lib.FpmError("Net.run: wrong-result timing probe(s) %s are switched on (ops.set_tuning); switch "
                           "them off before computing outputs" % ops.timing_probes_on())
        dev = bt.device
        B, n1max, n2max = bt.B, bt.n1max, bt.n2max
        parts = self._parts(bt, chunks)
        t0, t0c = time.perf_counter(), time.thread_time()
        device_lsa = self.lsa_mode == "device"
        graphed = self._graphed(parts, keep_feats)
        if not device_lsa and (self._pinned is None or self._pinned.shape != (B, n1max, n2max)):
            self._pinned = torch.empty((B, n1max, n2max), dtype=torch.float32, pin_memory=True)
            self._assign_pinned = torch.empty((B, n1max), dtype=torch.int32, pin_memory=True)
        main = torch.cuda.current_stream(dev)
        if graphed:
            gs = self._graph_state(bt, parts, dev)
            o, min_pt, gt_ks = gs["o"], gs["min_pt"], gs["gt_ks"]
        else:
            o = self._alloc_outputs(B, n1max, n2max, dev, k_f64=self._k_f64(bt))
            min_pt = torch.minimum(bt.n1, bt.n2).to(torch.float32)
            gt_ks = min_pt.clone()
        if gt_perm is not None:
            gt_ks.copy_(torch.as_tensor(gt_perm).to(dev).reshape(B, -1).sum(-1).to(torch.float32))
        elif graphed:
            gt_ks.copy_(min_pt)        # synthetic pairs: identity ground truth
        # ShardedNet: device threads enqueue one at a time (their HIP calls contend otherwise)
        lk = self._enqueue_lock
        if lk is not None:
            lk.acquire()
        try:
            ev_start = torch.cuda.Event(enable_timing=True)
            ev_start.record(main)
            self._mark("run_start")
            if graphed:
                gs["prologue"].replay()
                gc, xop, col, pre = gs["pro_out"]
            else:
                pro = self._prologue_replay(bt, parts, dev)
                gc, xop, col, pre = pro if pro is not None else self._prologue(bt, parts, cast=len(parts) > 1)
            ev_coef = torch.cuda.Event()
            ev_coef.record(main)
            streams = self._streams(dev) if (len(parts) > 1 and self.n_streams > 1) else [main]
            for st in streams:
                if st is not main:
                    st.wait_event(ev_coef)
            outs, done, plan_ev = [], [], []
            # copy deferral (plans computed per chunk only): chunk c's D2H waits for the plans of chunk
            # c + 2 (same stream)
            lag = 2 if (self.copy_defer and pre is None and len(parts) > 2 and len(streams) == 2 and not device_lsa
                        and not (self.zero_copy >= 2 and not graphed)) else 0
            events = [None] * len(parts)
            # host work units (pairs whose ds_mat lands together): one per chunk, or the tail groups
            # of a one-chunk forward (_tail_ranges) -> (chunk, unit part, b0, b1, D2H event)
            units = []
            split_tail = (len(parts) == 1 and not graphed and not device_lsa and not keep_feats and not self.compute_ke
                          and len(self._tail_ranges(0, B)) > 1)

            # zero-copy (FPM_ZERO_COPY 1: the tail groups of one-chunk forwards, 2: every chunk): the soft
            # top-k kernel writes the Hungarian's pinned rows itself -- no blit-kernel D2H, whose
            # workgroups slowed the kernels running beside it ~3x (round-5 trace of the 128-pair forward)
            zc_tail = split_tail and self.zero_copy >= 1
            zc_all = (not graphed and not device_lsa and not split_tail and self.zero_copy >= 2)

            def tail_unit(view, sb0, sb1):
                if zc_tail:
                    evt = torch.cuda.Event(enable_timing=True, blocking=True)
                    evt.record(torch.cuda.current_stream(dev))
                    units.append((0, view, sb0, sb1, evt))
                    return
                evt = torch.cuda.Event()
                evt.record(torch.cuda.current_stream(dev))
                units.append((0, view, sb0, sb1, self._enqueue_copy(dev, sb0, sb1, o, evt)))
            for c, part in enumerate(parts):
                st = streams[c % len(streams)]
                b0, b1 = (0, B) if part is bt else part.pair_range     # a chunk's range inside bt
                with torch.cuda.stream(st):
                    if graphed:
                        gpl, gst, _ = gs["chunks"][c]
                        if gpl is not None:
                            gpl.replay()
                    else:
                        pl = pre[c] if pre is not None else self.plans(part)
                    if lag:
                        evp = torch.cuda.Event()
                        evp.record(st)
                        plan_ev.append(evp)
                    if graphed:
                        gst.replay()
                        outs.append(None)
                    else:
                        outs.append(self._stage_a(part, b0, b1, o, keep_feats, gt_ks, min_pt, gc, col=col, xop=xop,
                                                  plans=pl, tail=tail_unit if split_tail else None,
                                                  zc=zc_tail or zc_all))
                    if split_tail:
                        continue
                    if device_lsa:
                        # the Hungarian kernel is latency-bound (one wave per pair): run it and the
                        # selection / classifier on a side stream so the next chunks' GPU stages are not
                        # queued behind it
                        ev = torch.cuda.Event(enable_timing=True)
                        ev.record(st)
                        side = self._lsa_streams(dev)[c % 2]
                        side.wait_event(ev)
                        with torch.cuda.stream(side):
                            self._stage_c_device(part, b0, b1, o)
                        events[c] = ev
                        continue
                    if zc_all:
                        ev = torch.cuda.Event(enable_timing=True, blocking=True)
                        ev.record(st)
                        events[c] = ev
                        continue
                    ev = torch.cuda.Event()
                    ev.record(st)
                    done.append((b0, b1, ev))
                if zc_all:
                    continue
                if not lag:
                    events[c] = self._enqueue_copy(dev, b0, b1, o, ev)
                elif c >= lag:
                    pb0, pb1, pdone = done[c - lag]
                    events[c - lag] = self._enqueue_copy(dev, pb0, pb1, o, pdone, after=plan_ev[c])
            if lag:
                for c in range(max(0, len(parts) - lag), len(parts)):
                    pb0, pb1, pdone = done[c]
                    events[c] = self._enqueue_copy(dev, pb0, pb1, o, pdone)
            if not split_tail:
                units = [(c, part, *((0, B) if part is bt else part.pair_range), events[c])
                         for c, part in enumerate(parts)]
            t_enq, t_enqc = time.perf_counter(), time.thread_time()
        finally:
            if lk is not None:
                lk.release()
        # the k losses need only k_prob (ngm.py:457-469): queued now on the last chunk's stream behind
        # every chunk's GPU stage, so their small kernels run while the host waits for the Hungarian
        # instead of after it (not on main: main carries stage C, which must not wait for them)
        last_st = streams[(len(parts) - 1) % len(streams)]
        for st in streams:
            if st is not last_st:
                last_st.wait_stream(st)
        losses = {}
        with torch.cuda.stream(last_st):
            if self.regression:
                losses["ks_loss"] = F.mse_loss(o["k_prob"], gt_ks / min_pt) * self.k_factor
                losses["ks_error"] = F.l1_loss(o["k_prob"] * min_pt, gt_ks)
            else:
                losses["ks_loss"] = 0.0
                losses["ks_error"] = 0.0
            if label is None:
                losses["cls_loss"] = torch.zeros((), device=dev)    # a fill kernel, not a synchronous H2D
        if getattr(self, "_sc_done", None) is not None:
            self._sc_done.synchronize()
            self._sc_done = None
        t_lsa, t_first = 0.0, None
        timeline = []      # per chunk: host ms (from t0) when its ds_mat had landed / its stage C was queued
        pending = []       # chunks whose Hungarian is queued on the LSA workers (lsa_async)

        # stage C (selection + classifier) on the forward's main stream, idle while the chunk streams
        # run, behind the unit's D2H event (which follows the unit's whole GPU stage): it overlaps the
        # later chunks' GPU stages.  Queued behind its chunk's own stream it waited for every later
        # chunk's GPU stage (all chunks are enqueued up front) and ran at the end of the forward
        # (~1.3 ms at C3, round-5 stage timeline).  No extra stream: hardware queues are few.
        sc = main if (not device_lsa and self.stagec_stream) else None
        unit_ev = {(u[2], u[3]): u[4] for u in units}
        unit_st = {(u[2], u[3]): streams[u[0] % len(streams)] for u in units}

        def stage_c_stream(b0_, b1_):
            if sc is None:                      # FPM_STAGEC_STREAM=0: the chunk's own stream
                return torch.cuda.stream(unit_st[(b0_, b1_)])
            sc.wait_event(unit_ev[(b0_, b1_)])
            return torch.cuda.stream(sc)

        def finish(entry, assign):
            c_, part_, b0_, b1_, tk, t_rdy_ = entry
            with stage_c_stream(b0_, b1_):
                self._stage_c(part_, b0_, b1_, o, assign=assign)
            timeline.append((round((t_rdy_ - t0) * 1e3, 3), round((time.perf_counter() - t0) * 1e3, 3)))
            return tk.seconds

        def drain_ready():
            # stage C of every queued unit (in order) whose Hungarian has finished
            nonlocal t_lsa
            done_any = False
            while pending:
                a = ops.lsa_wait(pending[0][4], block=False)
                if a is None:
                    break
                t_lsa += finish(pending.pop(0), a)
                done_any = True
            return done_any

        try:
            for c, part, b0, b1, ev in units:
                if device_lsa:
                    break
                if sc is not None and self.lsa_async and len(units) > 1:
                    # while this unit's D2H is in flight, queue the stage C of earlier units as soon as
                    # their Hungarian finishes (a blocking wait here held it back until this unit landed)
                    while not ev.query():
                        if not drain_ready():
                            time.sleep(5e-5)
                ev.synchronize()
                t_rdy = time.perf_counter()
                t_first = t_first or t_rdy
                if self.lsa_async and len(units) > 1:
                    # queue this chunk's pairs behind the earlier chunks' on the workers, then run the
                    # selection / classifier of every earlier chunk whose Hungarian has finished
                    tk = ops.lsa_submit(self._pinned[b0:b1], part.n_host[0], part.n_host[1], self.lsa_threads, b0=b0,
                                        out=self._assign_pinned[b0:b1])
                    pending.append((c, part, b0, b1, tk, t_rdy))
                    if sc is not None:
                        drain_ready()
                    else:
                        while len(pending) > 1:
                            a = ops.lsa_wait(pending[0][4], block=False)
                            if a is None:
                                break
                            t_lsa += finish(pending.pop(0), a)
                    continue
                with stage_c_stream(b0, b1):
                    t_lsa += self._stage_c(part, b0, b1, o)
                timeline.append((round((t_rdy - t0) * 1e3, 3), round((time.perf_counter() - t0) * 1e3, 3)))
            while pending:
                t_lsa += finish(pending[0], ops.lsa_wait(pending[0][4]))
                pending.pop(0)
        except BaseException:
            # a failing wait (infeasible / NaN pair) or an interrupt: every queued batch must finish
            # before its cost rows, pair sizes and assignment buffers can be dropped or reused
            ops.lsa_drain([p[4] for p in pending])
            torch.cuda.synchronize(dev)
            raise
        for st in streams:
            if st is not main:
                main.wait_stream(st)
        if sc is not None:
            if sc is not main:
                main.wait_stream(sc)
            # the next forward's Hungarian rewrites the pinned assignment rows only after this
            # forward's last H2D of them has run (run() waits on this event before its LSA)
            self._sc_done = torch.cuda.Event()
            self._sc_done.record(sc)
        if device_lsa:
            for st in self._lsa_streams(dev):
                main.wait_stream(st)
            bad = torch.nonzero(o["_lsa_status"]).view(-1)
            if bad.numel():
                raise RuntimeError("hungarian: pair %d is infeasible or has NaN/-inf costs" % int(bad[0]))
        res = {k: v for k, v in o.items() if not k.startswith("_")}
        if graphed:
            for k in ("ds_mat", "perm_mat", "k_prob", "cls_logits", "cls_prob", "sk_steps"):
                res[k] = o[k].clone()
        elif len(outs) == 1 or keep_feats:
            for k in outs[0]:
                if k not in ("s", "ss"):
                    res[k] = outs[0][k] if len(outs) == 1 else torch.cat([r[k] for r in outs])
        logits = res["cls_logits"]
        res.update(losses)
        if label is not None:
            res["cls_loss"] = F.binary_cross_entropy_with_logits(logits, torch.as_tensor(label).to(dev).view(-1).float())
        # GPU time of the stages before the Hungarian (all chunks), from events on the streams
        self.last_timing = dict(gpu_stage_s=ev_start.elapsed_time(units[-1][4]) / 1e3, lsa_s=t_lsa,
                                first_chunk_wait_s=(t_first or t0) - t0, chunks=len(parts), graphs=graphed,
                                host_units=len(units),
                                enqueue_s=t_enq - t0, enqueue_cpu_s=t_enqc - t0c, total_s=time.perf_counter() - t0,
                                chunk_timeline_ms=timeline)
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
