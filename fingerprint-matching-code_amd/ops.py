"""Thin torch-tensor wrappers over the C-ABI (``include/fpm.h``).

Every op takes device tensors, checks shapes/dtypes on the host, and launches on the current
torch stream.  Outputs are caller-allocated (``torch.empty`` on the tensor's device).  There is
no CPU fallback: a CPU tensor or a missing library raises.
"""
import ctypes

import torch

from . import _lib

F32, BF16 = 0, 1
EPI_STORE, EPI_RELU, EPI_TANH, EPI_AFFINITY, EPI_HALF_AFFINITY = 0, 1, 2, 3, 4
EPI_NORM_OUT = 6


def _p(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream(t=None):
    dev = t.device if t is not None else torch.device("cuda")
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.FpmError("fpm op called with a CPU tensor: the HIP path has no CPU fallback")


def _shape(t, shape, what):
    """Host-side operand check before a launch: ``t`` must cover ``shape`` exactly."""
    if t is not None and tuple(t.shape) != tuple(int(x) for x in shape):
        raise _lib.FpmError("%s: tensor of shape %s where %s is required" % (what, tuple(t.shape), tuple(shape)))


def _code(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise _lib.FpmError("unsupported operand dtype %s" % t.dtype)


def sinkhorn(s, n1, n2, iters, tau, dummy_row=True, out=None, n1max=None, n2max=None):
    """pygm-style log Sinkhorn on the (n1max, n2max) box of each pair.  ``s`` may be any strided
    3-D view (B, n1max, n2max); ``out`` likewise (allocated contiguous if None)."""
    _dev(s, n1, n2)
    B = s.shape[0]
    n1max = n1max or s.shape[1]
    n2max = n2max or s.shape[2]
    if out is None:
        out = torch.empty(B, n1max, n2max, device=s.device, dtype=torch.float32)
    _shape(out, (B, n1max, n2max), "sinkhorn out")
    _shape(n1, (B,), "sinkhorn n1")
    _shape(n2, (B,), "sinkhorn n2")
    # boxes over 256: the streaming kernel's split form needs a workspace of its own per call (exchange
    # slots + arrival counters; allocated on the caller's stream, so concurrent streams never share one)
    wsb = int(_lib.load().fpm_sinkhorn_ws_bytes(B, n1max, n2max)) if max(n1max, n2max) > 256 else 0
    ws = torch.empty(wsb, device=s.device, dtype=torch.uint8) if wsb > 0 else None
    _lib.call("fpm_sinkhorn_log_fwd_ws", _p(s), s.stride(0), s.stride(1), s.stride(2), _p(out), out.stride(0),
              out.stride(1), out.stride(2), _p(n1), _p(n2), B, n1max, n2max, int(iters), float(tau),
              int(bool(dummy_row)), _p(ws), wsb, _stream(s))
    return out


def soft_topk_fwd(ss, n1, n2, k, iters=10, tau=0.01, out=None, steps=None, out_host=None):
    """``out_host``: optional pinned host tensor written by the kernel as well (zero-copy D2H of
    ds_mat for the host Hungarian)."""
    _dev(ss, n1, n2, k)
    B, n1max, n2max = ss.shape
    if out is None:
        out = torch.empty(B, n1max, n2max, device=ss.device, dtype=torch.float32)
    _shape(out, (B, n1max, n2max), "soft_topk out")
    for t, w in ((n1, "n1"), (n2, "n2"), (k, "k"), (steps, "steps")):
        _shape(t, (B,), "soft_topk " + w)
    if out_host is not None and (out_host.is_cuda or not out_host.is_pinned() or tuple(out_host.shape) != (B, n1max, n2max)):
        raise _lib.FpmError("soft_topk: out_host must be a pinned host tensor of shape (B, n1max, n2max)")
    _lib.call("fpm_soft_topk_fwd", _p(ss), ss.stride(0), ss.stride(1), _p(n1), _p(n2), _p(k), B, n1max, n2max,
              int(iters), float(tau), _p(out), out.stride(0), out.stride(1), _p(steps), _p(out_host),
              out_host.stride(0) if out_host is not None else 0, out_host.stride(1) if out_host is not None else 0,
              _stream(ss))
    return out


def topk_select(ds, assign, k, lsa_out=None, out=None):
    _dev(ds, assign, k)
    B, n1max, n2max = ds.shape
    _shape(assign, (B, n1max), "topk_select assign")
    _shape(k, (B,), "topk_select k")
    _shape(out, (B, n1max, n2max), "topk_select out")
    _shape(lsa_out, (B, n1max, n2max), "topk_select lsa_out")
    perm = out if out is not None else torch.empty(B, n1max, n2max, device=ds.device, dtype=torch.float32)
    _lib.call("fpm_topk_select", _p(ds), ds.stride(0), ds.stride(1), _p(assign), assign.stride(0), _p(k), B,
              n1max, n2max, _p(perm), perm.stride(0), perm.stride(1), _p(lsa_out),
              lsa_out.stride(0) if lsa_out is not None else 0, lsa_out.stride(1) if lsa_out is not None else 0,
              _stream(ds))
    return perm


def profiling():
    """True while the library's HIP-event profiling of the product GEMM is on (fpm_profile_enable)."""
    return bool(_lib.load().fpm_profile_enabled())


_TUNING_GEN = [0]


def set_tuning(key, value):
    """Kernel-variant switch (fpm_set_tuning, include/fpm.h lists the keys).  Returns the previous
    value.  Every call bumps ``tuning_generation()`` (captured HIP graphs bake the variant in)."""
    prev = int(_lib.load().fpm_set_tuning(key.encode(), int(value)))
    if prev < 0:
        raise _lib.FpmError(_lib.load().fpm_last_error().decode(errors="replace"))
    _TUNING_GEN[0] += 1
    if key in WRONG_RESULT_PROBES:
        if int(value):
            _PROBES_ON.add(key)
        else:
            _PROBES_ON.discard(key)
    return prev


# timing probes whose results are wrong (gated by FPM_TIMING_PROBES=1 in the library); Net.run
# refuses to produce outputs while one of them is on
WRONG_RESULT_PROBES = ("gnn_mlp_off",)
_PROBES_ON = set()


def timing_probes_on():
    """Wrong-result timing probes currently switched on through ``set_tuning``."""
    return sorted(_PROBES_ON)


def tuning_generation():
    """Number of ``set_tuning`` calls so far (part of Net's graph-cache key)."""
    return _TUNING_GEN[0]


def gemm(A, B, M, N, K, lda, ldb, batch=1, sA=0, sB=0, a_rows=None, epi=EPI_STORE, bias=None, out_f=None,
         out_t=None, ldc=None, sC=0, n1=None, n2=None):
    """C = epi(A @ B^T (+bias)); A: rows of length >= K (lda), B: N x K (ldb)."""
    _dev(A, B)
    code = _code(A)
    if _code(B) != code:
        raise _lib.FpmError("gemm: A and B dtypes differ")
    if out_t is not None and _code(out_t) != code:
        raise _lib.FpmError("gemm: out_t dtype must match operands")
    _lib.call("fpm_gemm", code, _p(A), lda, sA, _p(a_rows), _p(B), ldb, sB, int(M), int(N), int(K), int(batch),
              int(epi), _p(bias), _p(out_f), _p(out_t), ldc if ldc is not None else N, sC, _p(n1), _p(n2),
              _stream(A))


def coef_tanh(g, wT, bias, out):
    """out[b] = tanh(g[b] @ wT + bias): g (B, K) fp32 rows, wT (K, N) fp32 -> out (B, N) (fpm_coef_tanh)."""
    _dev(g, wT, bias, out)
    B, K = g.shape
    N = wT.shape[1]
    if wT.shape[0] != K or g.stride(1) != 1 or not wT.is_contiguous() or tuple(out.shape) != (B, N):
        raise _lib.FpmError("coef_tanh: shapes g (B, K), wT (K, N) contiguous, out (B, N) expected")
    _lib.call("fpm_coef_tanh", _p(g), g.stride(0), _p(wT), _p(bias), B, K, N, _p(out), out.stride(0), _stream(g))
    return out


def global_weights(w1, w2, out=None):
    """normalize_over_channels(cat(w1, w2)) per pair (ngm.py:262-268) -> (B, D1 + D2) fp32."""
    _dev(w1, w2)
    if w1.dtype != torch.float32 or w2.dtype != torch.float32 or w1.stride(1) != 1 or w2.stride(1) != 1:
        raise _lib.FpmError("global_weights: float32 rows with unit stride expected")
    B, D1 = w1.shape
    D2 = w2.shape[1]
    _shape(w2, (B, D2), "global_weights w2")
    if out is None:
        out = torch.empty(B, D1 + D2, device=w1.device, dtype=torch.float32)
    _shape(out, (B, D1 + D2), "global_weights out")
    _lib.call("fpm_global_weights", _p(w1), w1.stride(0), _p(w2), w2.stride(0), B, D1, D2, _p(out), out.stride(0),
              _stream(w1))
    return out


def split_bf16x3(x, Kp, out=None):
    """(rows, K) fp32 rows -> (rows, 3 * Kp) bf16 [hi | lo | hi] split operands (fpm_split_bf16x3)."""
    _dev(x)
    if x.dtype != torch.float32 or x.dim() != 2 or x.stride(1) != 1:
        raise _lib.FpmError("split_bf16x3: (rows, K) float32 rows with unit stride expected")
    rows, K = x.shape
    if out is None:
        out = torch.empty(rows, 3 * Kp, device=x.device, dtype=torch.bfloat16)
    _shape(out, (rows, 3 * Kp), "split_bf16x3 out")
    _lib.call("fpm_split_bf16x3", _p(x), x.stride(0), rows, K, int(Kp), _p(out), out.stride(0), _stream(x))
    return out


def split_weights_bf16x3(W, Kp):
    """(N, K) fp32 weights -> (N, 3 * Kp) bf16 [W_hi | W_hi | W_lo] (parameter packing, host side)."""
    N, K = W.shape
    Wp = torch.nn.functional.pad(W.float(), (0, Kp - K))
    hi = Wp.to(torch.bfloat16)
    lo = (Wp - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, hi, lo], dim=1).contiguous()


def cast_bf16(x, out=None):
    _dev(x)
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
    _lib.call("fpm_cast_bf16", _p(x), _p(out), x.numel(), _stream(x))
    return out


def spline_plan(src, dst, pseudo, num_nodes, nmax, max_graph_edges=0):
    """``max_graph_edges``: the largest per-graph edge count (host-known, e.g. from the batch's edge
    offsets) -> the per-graph plan kernels when it allows; 0 -> the global plan kernels."""
    _dev(src, dst, pseudo)
    E = src.numel()
    nbytes = _lib.load().fpm_spline_plan_bytes(E, num_nodes)
    ws = torch.empty(nbytes, device=src.device, dtype=torch.uint8)
    _lib.call("fpm_spline_plan_graphs", _p(src), _p(dst), _p(pseudo), E, num_nodes, nmax, int(max_graph_edges), _p(ws),
              nbytes, _stream(src))
    return ws


def spline_plan_jobs(parts, side, nmax):
    """The device job table of spline_plans_multi for ``parts`` (built once, cached while the first
    part lives; its host-to-device copy must not run inside a graph capture) -> tuple or None."""
    first = parts[0]
    dev = first.src[side].device
    key = (id(first), len(parts), side)
    store = _PLAN_JOBS.get(key)
    if store is not None and store[0]() is first:
        return store
    import weakref
    jobs, off, gstart = [], 0, 0
    for p in parts:
        E, nn = p.E[side], p.B * nmax
        if not (0 < p.max_graph_edges(side) <= 4096 and 26 <= nmax <= 1024 and p.B + 1 <= E):
            _PLAN_JOBS[key] = store = (weakref.ref(first), None)
            return store
        nbytes = int(_lib.load().fpm_spline_plan_bytes(E, nn))
        jobs.append([p.src[side].data_ptr(), p.dst[side].data_ptr(), p.pseudo[side].data_ptr(), E, nn, off,
                     (gstart << 32) | p.B])
        off += (nbytes + 255) // 256 * 256
        gstart += p.B
    if int(_lib.load().fpm_spline_plan_job_bytes()) != 56:
        raise _lib.FpmError("spline_plans_multi: PlanJob layout mismatch")
    table = torch.tensor(jobs, dtype=torch.int64).to(dev)
    sizes = [int(_lib.load().fpm_spline_plan_bytes(p.E[side], p.B * nmax)) for p in parts]
    store = (weakref.ref(first), table, [j[5] for j in jobs], sizes, off, gstart)
    _PLAN_JOBS[key] = store
    if len(_PLAN_JOBS) > 64:
        for k in [k for k, v in _PLAN_JOBS.items() if v[0]() is None]:
            del _PLAN_JOBS[k]
    return store


def spline_plans_multi(parts, side, nmax):
    """The spline plans of ``side`` for every sub-batch in ``parts`` (pipeline chunks of one batch)
    by one launch of each per-graph plan kernel (fpm_spline_plan_multi) -> list of plan workspaces
    (views into one allocation), each identical to spline_plan() of that sub-batch alone; None when
    some sub-batch needs the global plan kernels (graphs over 4096 edges, nmax outside [26, 1024])."""
    store = spline_plan_jobs(parts, side, nmax)
    if store[1] is None:
        return None
    _, table, offs, sizes, total, ngraphs = store
    ws = torch.empty(total, device=table.device, dtype=torch.uint8)
    _lib.call("fpm_spline_plan_multi", _p(table), len(parts), ngraphs, nmax, _p(ws), _stream(ws))
    return [ws[o:o + n] for o, n in zip(offs, sizes)]


_PLAN_JOBS = {}


def plan_csr(ws, E, num_nodes):
    """(dst_ptr, nbr_local) raw device pointers (ints) inside a plan workspace."""
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.call("fpm_spline_plan_csr", _p(ws), E, num_nodes, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def spline_y_ws(dtype_code, E, num_nodes, device):
    """Product-row scratch for spline_conv (shared by both layers of a side)."""
    nbytes = _lib.load().fpm_spline_y_bytes(dtype_code, E, num_nodes)
    return torch.empty(nbytes, device=device, dtype=torch.uint8)


def spline_conv(x_op, plan, E, num_nodes, nmax, nvalid, W, bias, y_ws, mode, xres=None, cscale=None, out_f=None,
                out_t=None, argmax=None):
    """W: (26, 768, 768) = spline cells [cell][out][in] then root^T.  argmax (num_nodes, 768) int32:
    optional per-channel max in-edge slots for spline_conv_bwd_data(..., rplan=, argmax=)."""
    _dev(x_op, plan, W, bias, y_ws)
    code = _code(x_op)
    if _code(W) != code or tuple(W.shape) != (26, 768, 768):
        raise _lib.FpmError("spline_conv: W must be (26, 768, 768) in the operand dtype")
    if argmax is not None:
        _shape(argmax, (num_nodes, 768), "spline_conv argmax")
        if argmax.dtype != torch.int32:
            raise _lib.FpmError("spline_conv: argmax must be int32")
        _lib.call("fpm_spline_conv_fwd_argmax", code, _p(x_op), _p(plan), E, num_nodes, nmax, _p(nvalid), _p(W),
                  _p(bias), _p(y_ws), y_ws.numel(), int(mode), _p(xres), _p(cscale), _p(out_f), _p(out_t),
                  _p(argmax), _stream(x_op))
        return
    _lib.call("fpm_spline_conv_fwd", code, _p(x_op), _p(plan), E, num_nodes, nmax, _p(nvalid), _p(W), _p(bias),
              _p(y_ws), y_ws.numel(), int(mode), _p(xres), _p(cscale), _p(out_f), _p(out_t), _stream(x_op))


def rows_bcast_scale(y, B, coef=None, out_f=None, out_t=None, split=0):
    """Shared-graph SplineConv output y (rows, 768) fp32 -> B pairs (out_f copies, out_t scaled by coef[b]);
    ``split`` 1 / 2: bf16 out_t rows of 2304 columns [hi | lo | hi] / [hi | hi | lo] (spline_conv's mode >> 1)."""
    _dev(y, coef, out_f, out_t)
    code = _code(out_t) if out_t is not None else F32
    _lib.call("fpm_rows_bcast_scale", code, _p(y), y.shape[0], int(B), _p(coef), _p(out_f), _p(out_t), int(split),
              _stream(y))


def edge_diff(x, src, dst):
    _dev(x, src, dst)
    E, D = src.numel(), x.shape[-1]
    out = torch.empty(E, D, device=x.device, dtype=torch.float32)
    _lib.call("fpm_edge_diff", _p(x), _p(src), _p(dst), E, D, _p(out), _stream(x))
    return out


def edge_diff_padded(x, src, dst, pair, row, nrows, cscale=None):
    """(nrows, D) zero-padded: out[row[e]] = (x[src[e]] - x[dst[e]]) * cscale[pair[e]]."""
    _dev(x, src, dst, pair, row)
    E, D = src.numel(), x.shape[-1]
    out = torch.zeros(nrows, D, device=x.device, dtype=torch.float32)
    _lib.call("fpm_edge_diff_padded", _p(x), _p(src), _p(dst), _p(pair), _p(row), _p(cscale), E, D, _p(out),
              _stream(x))
    return out


def gnn_layer(X, C, B, n1max, n2max, csr1, csr2, n1, n2, params, Xout, zbuf, vpart=None, cls_w=None, ord2=None):
    """``ord2``: optional (B, n2max) int32 block order of the graph-2 nodes (a schedule; same results)."""
    _dev(X, n1, n2, params, Xout, zbuf, vpart, cls_w, ord2)
    _shape(X, (B, C, n2max, n1max), "gnn_layer X")
    _shape(Xout, (B, 17, n2max, n1max), "gnn_layer Xout")
    _shape(zbuf, (B, n2max, n1max), "gnn_layer zbuf")
    _shape(vpart, (B, n2max, n1max), "gnn_layer vpart")
    _shape(ord2, (B, n2max), "gnn_layer ord2")
    _lib.call("fpm_kron_gnn_layer_fwd_ord", _p(X), C, B, n1max, n2max, ctypes.c_void_p(csr1[0]),
              ctypes.c_void_p(csr1[1]), ctypes.c_void_p(csr2[0]), ctypes.c_void_p(csr2[1]), _p(n1), _p(n2),
              _p(params), _p(Xout), _p(zbuf), _p(vpart), _p(cls_w), _p(ord2), _stream(X))


def node_classifier(X, B, n1max, n2max, w, b, out, vpart=None):
    _dev(X, w, b, out, vpart)
    _shape(X, (B, 17, n2max, n1max), "node_classifier X")
    _shape(out, (B, n1max, n2max), "node_classifier out")
    _shape(vpart, (B, n2max, n1max), "node_classifier vpart")
    _lib.call("fpm_node_classifier", _p(X), B, n1max, n2max, _p(w), _p(b), _p(vpart), _p(out), _stream(X))


def crossset_attn(cost, n2, Wv, mix1w, mix1b, mix2w, mix2b, out, split=False, stats=None):
    """``split``: out is (B * n1max, 768) bf16 [hi | lo | hi] rows (near-fp32 operand); ``stats``:
    optional (B * n1max, 16, 2) fp32 softmax (max, sum) per row and head (training)."""
    _dev(cost, n2, Wv, out)
    B, n1max, n2max = cost.shape
    _shape(out, (B * n1max, 768 if split else 256), "crossset_attn out")
    if split and out.dtype != torch.bfloat16:
        raise _lib.FpmError("crossset_attn: split rows are bf16")
    _shape(stats, (B * n1max, 16, 2), "crossset_attn stats")
    _lib.call("fpm_crossset_attn_fwd", 2 if split else _code(out), _p(cost), cost.stride(0), cost.stride(1), B, n1max, n2max,
              _p(n2), _p(Wv), Wv.shape[1], _p(mix1w), _p(mix1b), _p(mix2w), _p(mix2b), _p(out), _p(stats),
              _stream(cost))


def instnorm(in1, B, P, Cn, w, b, in2=None, nvalid=None, onehot_bias=None, out_f=None, out_t=None, gmax=None,
             eps=1e-5, ldt=0):
    """``ldt`` > Cn: out_t rows are ldt wide and columns [Cn, ldt) are written as zeros."""
    code = _code(out_t) if out_t is not None else F32
    ref = in1 if in1 is not None else w
    _lib.call("fpm_instnorm", code, _p(in1), _p(in2), B, P, Cn, _p(nvalid), _p(onehot_bias), _p(w), _p(b),
              float(eps), _p(out_f), _p(out_t), int(ldt), _p(gmax), _stream(ref))


def gemm_norm_max(A, Bw, M, N, K, lda, ldb, bias, res, nw, nb, gmax, P=256, eps=1e-5):
    """AFA-U block tail fused (fpm_gemm_norm_max): gmax[b][n] = max over the pair's P rows of
    InstanceNorm(res + A Bw^T + bias) * nw + nb; bf16 A / Bw, P = 256 or 128 rows per pair (one or
    two pairs per 256-row tile)."""
    _dev(A, Bw, res, gmax)
    _lib.call("fpm_gemm_norm_max", _p(A), int(lda), _p(Bw), int(ldb), int(M), int(N), int(K), _p(bias), _p(res),
              int(res.stride(0)), _p(nw), _p(nb), float(eps), int(P), _p(gmax), _stream(A))
    return gmax


def gemm_norm_out(A, Bw, M, N, K, lda, ldb, bias, nw, nb, out_f, out_t=None, ldt=0, P=256, eps=1e-5):
    """AFA-U block head fused (fpm_gemm_norm_out): out_f = InstanceNorm over each pair's P rows of
    (A Bw^T + bias) * nw + nb, out_t its bf16 copy (row stride ldt, zero columns [N, ldt))."""
    _dev(A, Bw, out_f)
    _lib.call("fpm_gemm_norm_out", _p(A), int(lda), _p(Bw), int(ldb), int(M), int(N), int(K), _p(bias), _p(nw),
              _p(nb), float(eps), int(P), _p(out_f), int(out_f.stride(0)), _p(out_t),
              int(ldt or (out_t.stride(0) if out_t is not None else 0)), _stream(A))
    return out_f


def affinity(X1, X2, w, A_w, A_b, n1, n2, half=False, out=None):
    """InnerProductWithWeightsAffinity._forward for a batch of pairs (fpm_affinity_fwd,
    affinity_layer.py:11-19): X1 (B, n1max, d), X2 (B, n2max, d), w (B, kw) fp32 device tensors,
    A_w (d, kw), A_b (d,) -> K (B, n1max, n2max) = softplus((X1 o tanh(A_w w + A_b)) X2^T) - 0.5 on
    each pair's valid block (``half``: 0.5 * (...), the edge affinity), 0 elsewhere."""
    _dev(X1, X2, w, A_w, A_b, n1, n2)
    for t in (X1, X2, w, A_w, A_b):
        if t.dtype != torch.float32:
            raise _lib.FpmError("affinity: float32 operands expected")
    B, n1max, d = X1.shape
    n2max = X2.shape[1]
    kw = w.shape[1]
    _shape(X2, (B, n2max, d), "affinity X2")
    _shape(w, (B, kw), "affinity w")
    _shape(A_w, (d, kw), "affinity A_w")
    _shape(n1, (B,), "affinity n1")
    _shape(n2, (B,), "affinity n2")
    X1, X2, w, A_w = (t.contiguous() for t in (X1, X2, w, A_w))
    if out is None:
        out = torch.empty(B, n1max, n2max, device=X1.device, dtype=torch.float32)
    _shape(out, (B, n1max, n2max), "affinity out")
    nws = int(_lib.load().fpm_affinity_ws_floats(B, n1max, d))
    ws = torch.empty(max(nws, 1), device=X1.device, dtype=torch.float32)
    _lib.call("fpm_affinity_fwd", _p(X1), d, _p(X2), d, _p(w), kw, _p(A_w), _p(A_b), B, n1max, n2max, d,
              _p(n1.to(torch.int32)), _p(n2.to(torch.int32)), 1 if half else 0, _p(out), out.stride(1), _p(ws), nws,
              _stream(X1))
    return out


_RANGE = {"bad": None, "calls": 0}


def _range_every():
    import os
    return int(os.environ.get("FPM_LOSS_CHECK_EVERY", "1"))


def perm_loss_fwd(ds, gt, n1, n2, check_range=None):
    """PermutationLoss (src/loss_func.py:26-59) of device ds / gt (B, n1max, n2max views with unit
    column stride), n1 / n2 (B,) int32 device -> 0-d fp32 device tensor (fpm_perm_loss_fwd).  Each
    pair's block is clamped to the padded box like the reference's slice.

    Range check (the reference asserts 0 <= x <= 1 on both tensors, loss_func.py:42-47): entries of
    each pair's VALID block outside [0, 1] or NaN raise FpmError (the padding, which the reference's
    assert also covers, is not read: the device ds_mat is 0 there by construction).  The reference's
    assert reads the device on every call; here ``check_range`` (None: FPM_LOSS_CHECK_EVERY, default
    1) = 1 does the same, N > 1 accumulates the per-pair flags on the device and reads them every N-th
    call (the error names the calls since the last read), 0 / False skips the check."""
    _dev(ds, gt, n1, n2)
    B, n1max, n2max = ds.shape
    if ds.stride(2) != 1 or gt.stride(2) != 1 or tuple(gt.shape) != tuple(ds.shape):
        raise _lib.FpmError("perm_loss: ds / gt (B, n1max, n2max) with unit column stride expected")
    every = _range_every() if check_range is None else int(check_range)
    ws = torch.empty(B, device=ds.device, dtype=torch.float32)
    bad = torch.zeros(B, device=ds.device, dtype=torch.int32) if every > 0 else None
    out = torch.empty((), device=ds.device, dtype=torch.float32)
    _lib.call("fpm_perm_loss_fwd", _p(ds), ds.stride(0), ds.stride(1), _p(gt), gt.stride(0), gt.stride(1), _p(n1), _p(n2),
              B, n1max, n2max, _p(ws), _p(bad), _p(out), _stream(ds))
    if every <= 0:
        return out
    if every == 1:
        if int(bad.sum()):
            pairs = bad.nonzero().view(-1).tolist()
            raise _lib.FpmError("perm_loss: ds_mat / gt_perm_mat entries outside [0, 1] (or NaN) in pair(s) %s "
                                "(the reference asserts 0 <= x <= 1, loss_func.py:42-47)" % pairs[:8])
        return out
    acc = _RANGE["bad"]
    tot = bad.sum()
    _RANGE["bad"] = tot if acc is None or acc.device != tot.device else acc + tot
    _RANGE["calls"] += 1
    if _RANGE["calls"] >= every:
        n, calls = int(_RANGE["bad"]), _RANGE["calls"]
        _RANGE["bad"], _RANGE["calls"] = None, 0
        if n:
            raise _lib.FpmError("perm_loss: %d pair(s) with ds_mat / gt_perm_mat entries outside [0, 1] (or NaN) "
                                "in the last %d loss calls (the reference asserts 0 <= x <= 1, "
                                "loss_func.py:42-47)" % (n, calls))
    return out


def perm_loss_bwd(ds, gt, n1, n2, g):
    """d loss / d ds of perm_loss_fwd for the loss gradient ``g`` (0-d device tensor) -> contiguous
    (B, n1max, n2max) fp32."""
    _dev(ds, gt, n1, n2, g)
    B, n1max, n2max = ds.shape
    ws = torch.empty(1, device=ds.device, dtype=torch.float32)
    dds = torch.empty(B, n1max, n2max, device=ds.device, dtype=torch.float32)
    _lib.call("fpm_perm_loss_bwd", _p(ds), ds.stride(0), ds.stride(1), _p(gt), gt.stride(0), gt.stride(1), _p(n1), _p(n2),
              B, n1max, n2max, _p(g.float().contiguous()), _p(ws), _p(dds), _stream(ds))
    return dds


def gemm_x3out(A, Bw, M, N, K, Kp, epi=EPI_STORE, bias=None, out_t3=None, out_f=None, nw=None, nb=None, P=256,
               eps=1e-5):
    """C = epi(A Bw^T + bias) (bf16 A / Bw, fp32 accumulation) written as split bf16 rows
    out_t3 = [hi | lo | hi] (segment Kp, zero K padding; = split_bf16x3 of the fp32 C) and, if
    ``out_f`` is given, fp32 rows.  epi: EPI_STORE, EPI_RELU or EPI_NORM_OUT (instance norm over
    each pair's P = 256 or 128 rows, nw / nb) -- fpm_gemm_x3out.  Returns out_t3."""
    _dev(A, Bw, out_t3, out_f)
    for t, w in ((A, "A"), (Bw, "B")):
        if t.dtype != torch.bfloat16 or t.dim() != 2 or t.stride(1) != 1:
            raise _lib.FpmError("gemm_x3out: %s must be (rows, K) bf16 rows with unit stride" % w)
    if A.shape[0] < M or A.shape[1] < K or Bw.shape[0] != N or Bw.shape[1] < K:
        raise _lib.FpmError("gemm_x3out: operand shapes %s x %s do not cover M=%d N=%d K=%d"
                            % (tuple(A.shape), tuple(Bw.shape), M, N, K))
    if out_t3 is None:
        out_t3 = torch.empty(M, 3 * Kp, device=A.device, dtype=torch.bfloat16)
    if out_t3.dtype != torch.bfloat16 or out_t3.shape[0] != M or out_t3.stride(1) != 1 or out_t3.shape[1] < 3 * Kp:
        raise _lib.FpmError("gemm_x3out: out_t3 must be (M, >= 3 Kp) bf16")
    if out_f is not None and (out_f.dtype != torch.float32 or out_f.shape[0] != M or out_f.shape[1] < N):
        raise _lib.FpmError("gemm_x3out: out_f must be (M, >= N) float32")
    _lib.call("fpm_gemm_x3out", _p(A), int(A.stride(0)), _p(Bw), int(Bw.stride(0)), int(M), int(N), int(K), int(epi),
              _p(bias), _p(nw), _p(nb), float(eps), int(P), _p(out_f), int(out_f.stride(0)) if out_f is not None else 0,
              _p(out_t3), int(out_t3.stride(0)), int(Kp), _stream(A))
    return out_t3


def afau_head(gr, gc, B, E, r0w, r0b, r2w, r2b, c0w, c0b, c2w, c2b, ks):
    _lib.call("fpm_afau_head", _p(gr), _p(gc), B, E, _p(r0w), _p(r0b), _p(r2w), _p(r2b), _p(c0w), _p(c0b),
              _p(c2w), _p(c2b), _p(ks), _stream(gr))


# ---- fp64 k chain (csrc/precise.hip): Kp -> GNN layers -> readout -> final Sinkhorn -> AFA-U -------
def _f64(*ts):
    for t in ts:
        if t is not None and t.dtype != torch.float64:
            raise _lib.FpmError("fp64 k-chain op: float64 tensor expected, got %s" % t.dtype)


def gnn_layer_f64(X, C, B, n1max, n2max, csr1, csr2, n1, n2, params, Xout, zbuf):
    """PYGNNLayer in fp64: X (B, C, n2max, n1max) fp32 Kp for C = 1, the fp64 state for C = 17 ->
    Xout[:, 0:16] (fp64) and zbuf (B, n2max, n1max) fp64 (fpm_kron_gnn_layer_fwd_f64)."""
    _dev(X, n1, n2, params, Xout, zbuf)
    _shape(X, (B, C, n2max, n1max), "gnn_layer_f64 X")
    _shape(Xout, (B, 17, n2max, n1max), "gnn_layer_f64 Xout")
    _shape(zbuf, (B, n2max, n1max), "gnn_layer_f64 zbuf")
    _f64(Xout, zbuf)
    if not (X.is_contiguous() and Xout.is_contiguous() and zbuf.is_contiguous()):
        raise _lib.FpmError("gnn_layer_f64: contiguous tensors expected")
    x64 = X.dtype == torch.float64
    if x64 != (C == 17) or (not x64 and X.dtype != torch.float32):
        raise _lib.FpmError("gnn_layer_f64: layer 0 reads fp32 Kp (C = 1), later layers the fp64 state (C = 17)")
    _lib.call("fpm_kron_gnn_layer_fwd_f64", _p(X), int(x64), C, B, n1max, n2max, ctypes.c_void_p(csr1[0]),
              ctypes.c_void_p(csr1[1]), ctypes.c_void_p(csr2[0]), ctypes.c_void_p(csr2[1]), _p(n1), _p(n2),
              _p(params), _p(Xout), _p(zbuf), _stream(X))


def sinkhorn_f64(s, n1, n2, iters, tau, dummy_row=True, out=None, out32=None):
    """pygm log Sinkhorn in fp64 on each pair's valid block of the (n1max, n2max) box: ``s`` any
    strided fp32 / fp64 3-D view, ``out`` an fp64 view (allocated when None and ``out32`` is None),
    ``out32`` an optional fp32 copy.  Boxes up to 128 x 128."""
    _dev(s, n1, n2, out, out32)
    B, n1max, n2max = s.shape
    if out is None and out32 is None:
        out = torch.empty(B, n1max, n2max, device=s.device, dtype=torch.float64)
    _shape(out, (B, n1max, n2max), "sinkhorn_f64 out")
    _shape(out32, (B, n1max, n2max), "sinkhorn_f64 out32")
    _shape(n1, (B,), "sinkhorn_f64 n1")
    _shape(n2, (B,), "sinkhorn_f64 n2")
    _f64(out)
    if out32 is not None and out32.dtype != torch.float32:
        raise _lib.FpmError("sinkhorn_f64: out32 must be float32")
    if s.dtype not in (torch.float32, torch.float64):
        raise _lib.FpmError("sinkhorn_f64: s must be float32 or float64")
    st = lambda t: (t.stride(0), t.stride(1), t.stride(2)) if t is not None else (0, 0, 0)
    _lib.call("fpm_sinkhorn_log_fwd_f64", _p(s), int(s.dtype == torch.float64), *st(s), _p(out), *st(out), _p(out32),
              *st(out32), _p(n1), _p(n2), B, n1max, n2max, int(iters), float(tau), int(bool(dummy_row)), _stream(s))
    return out


def node_classifier_f64(X, B, n1max, n2max, w, b, s64, s32=None):
    """s = classifier(emb) (ngm.py:368-369) from the fp64 state: s64 (B, n1max, n2max) fp64 and
    optionally its fp32 copy."""
    _dev(X, w, b, s64, s32)
    _shape(X, (B, 17, n2max, n1max), "node_classifier_f64 X")
    _shape(s64, (B, n1max, n2max), "node_classifier_f64 s64")
    _shape(s32, (B, n1max, n2max), "node_classifier_f64 s32")
    _f64(X, s64)
    for t in (X, s64, s32):
        if t is not None and not t.is_contiguous():
            raise _lib.FpmError("node_classifier_f64: contiguous tensors expected")
    _lib.call("fpm_node_classifier_f64", _p(X), B, n1max, n2max, _p(w), _p(b), _p(s64), _p(s32), _stream(X))


def crossset_attn_row_f64(cost, n2, Wv, mix1w, mix1b, mix2w, mix2b, out):
    """The AFA-U row block's cross-set attention (R0 = 0) in fp64: cost (B, n1max, n2max) fp64 with
    unit column stride -> out (B * n1max, 256) fp64."""
    _dev(cost, n2, Wv, out)
    _f64(cost, Wv, mix1w, mix1b, mix2w, mix2b, out)
    B, n1max, n2max = cost.shape
    _shape(out, (B * n1max, 256), "crossset_attn_row_f64 out")
    if cost.stride(2) != 1 or not Wv.is_contiguous() or not out.is_contiguous():
        raise _lib.FpmError("crossset_attn_row_f64: unit-stride cost rows, contiguous Wv / out expected")
    _lib.call("fpm_crossset_attn_row_f64", _p(cost), cost.stride(0), cost.stride(1), B, n1max, n2max, _p(n2), _p(Wv),
              Wv.shape[1], _p(mix1w), _p(mix1b), _p(mix2w), _p(mix2b), _p(out), _stream(cost))


def gemm_f64(A, W, bias=None, relu=False, out=None):
    """out = act(A @ W^T + bias) in fp64 (fpm_gemm_f64): A (M, K), W (N, K)."""
    _dev(A, W, bias, out)
    _f64(A, W, bias, out)
    M, K = A.shape
    N = W.shape[0]
    if W.shape[1] != K or A.stride(1) != 1 or W.stride(1) != 1:
        raise _lib.FpmError("gemm_f64: A (M, K), W (N, K) with unit column stride expected")
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=torch.float64)
    _shape(out, (M, N), "gemm_f64 out")
    _lib.call("fpm_gemm_f64", _p(A), A.stride(0), _p(W), W.stride(0), _p(bias), _p(out), out.stride(0), M, N, K,
              int(bool(relu)), _stream(A))
    return out


def instnorm_f64(in1, B, P, Cn, w, b, in2=None, nvalid=None, onehot_bias=None, out=None, gmax=None, eps=1e-5):
    """AddAndInstanceNormalization (afau.py:154-176) in fp64 over each pair's P rows of Cn channels:
    x = in1 (+ in2), or the col block's one-hot + bias; out (B * P, Cn) and/or gmax (B, Cn)."""
    ref = in1 if in1 is not None else w
    _dev(ref, in2, nvalid, onehot_bias, w, b, out, gmax)
    _f64(in1, in2, onehot_bias, w, b, out, gmax)
    for t in (in1, in2, out):
        _shape(t, (B * P, Cn), "instnorm_f64 rows")
    _shape(gmax, (B, Cn), "instnorm_f64 gmax")
    _lib.call("fpm_instnorm_f64", _p(in1), _p(in2), B, P, Cn, _p(nvalid), _p(onehot_bias), _p(w), _p(b), float(eps),
              _p(out), _p(gmax), _stream(ref))


def afau_head_f64(gr, gc, cidx, B, E, r0w, r0b, r2w, r2b, c0w, c0b, c2w, c2b, ks):
    """ks = sigmoid((final_row(gr) + final_col(gc[cidx])) / 2) from fp64 pooled rows -> ks fp32."""
    _dev(gr, gc, cidx, ks)
    _f64(gr, gc, r0w, r0b, r2w, r2b, c0w, c0b, c2w, c2b)
    _shape(gr, (B, E), "afau_head_f64 gr")
    _shape(ks, (B,), "afau_head_f64 ks")
    if cidx is not None and (cidx.dtype != torch.int32 or tuple(cidx.shape) != (B,)):
        raise _lib.FpmError("afau_head_f64: cidx must be int32 (B,)")
    _lib.call("fpm_afau_head_f64", _p(gr), _p(gc), _p(cidx), B, E, _p(r0w), _p(r0b), _p(r2w), _p(r2b), _p(c0w),
              _p(c0b), _p(c2w), _p(c2b), _p(ks), _stream(gr))


def soft_topk_f64(ss, n1, n2, k, iters=10, tau=0.01, out=None, steps=None, out_host=None):
    """soft_topk(..., return_prob=True)[1] in fp64 from the fp64 ss (unit column stride) -> ds_mat
    fp32 (B, n1max, n2max); ``steps``: (B,) int32 steps taken incl. the while loop; ``out_host``: a
    pinned host copy written by the kernel too."""
    _dev(ss, n1, n2, k, out, steps)
    _f64(ss)
    B, n1max, n2max = ss.shape
    if ss.stride(2) != 1:
        raise _lib.FpmError("soft_topk_f64: ss rows with unit column stride expected")
    if out is None:
        out = torch.empty(B, n1max, n2max, device=ss.device, dtype=torch.float32)
    _shape(out, (B, n1max, n2max), "soft_topk_f64 out")
    for t, w in ((n1, "n1"), (n2, "n2"), (k, "k"), (steps, "steps")):
        _shape(t, (B,), "soft_topk_f64 " + w)
    if out.stride(2) != 1 or (out_host is not None and (out_host.is_cuda or not out_host.is_pinned()
                                                       or tuple(out_host.shape) != (B, n1max, n2max))):
        raise _lib.FpmError("soft_topk_f64: out with unit column stride, out_host pinned (B, n1max, n2max)")
    ws = torch.empty(2 * B * n1max * n2max, device=ss.device, dtype=torch.float64)
    _lib.call("fpm_soft_topk_fwd_f64", _p(ss), ss.stride(0), ss.stride(1), _p(n1), _p(n2), _p(k), B, n1max, n2max,
              int(iters), float(tau), _p(ws), ws.numel(), _p(out), out.stride(0), out.stride(1), _p(steps),
              _p(out_host), out_host.stride(0) if out_host is not None else 0,
              out_host.stride(1) if out_host is not None else 0, _stream(ss))
    return out


def match_cls(s, perm, w1, b1, bn1_sc, bn1_sh, w2, b2, bn2_sc, bn2_sh, fcw, fcb, logits=None, prob=None, dtype=F32):
    _dev(s, perm)
    if not (s.is_contiguous() and perm.is_contiguous()):
        raise _lib.FpmError("match_cls: s and perm must be contiguous")
    B, H, W = s.shape
    nws = _lib.load().fpm_match_cls_ws_floats(B, H, W)
    ws = torch.empty(max(int(nws), 1), device=s.device, dtype=torch.float32)
    logits = logits if logits is not None else torch.empty(B, device=s.device, dtype=torch.float32)
    prob = prob if prob is not None else torch.empty(B, device=s.device, dtype=torch.float32)
    _lib.call("fpm_match_cls_fwd", int(dtype), _p(s), _p(perm), B, H, W, _p(w1), _p(b1), _p(bn1_sc), _p(bn1_sh), _p(w2), _p(b2),
              _p(bn2_sc), _p(bn2_sh), _p(fcw), _p(fcb), _p(ws), _p(logits), _p(prob), _stream(s))
    return logits, prob


def feature_align(nodes, edges, P, n, nmax=None, ori_size=(320.0, 240.0), out=None, wglob=None, keep_ws=False):
    """Normalise both CNN maps over channels, bilinear-gather them at the keypoints
    (utils/feature_align.py) and concatenate -> X (B*nmax, C_n + C_e) fp32 with zero padding rows;
    also the global max-pooled edge feature (B, C_e).  Maps may be NCHW or channels_last.
    ``keep_ws``: also return the workspace (pixel norms) for feature_align_bwd."""
    _dev(nodes, edges, P, n)
    for t in (nodes, edges, P):
        if t.dtype != torch.float32:
            raise _lib.FpmError("feature_align: float32 maps and keypoints expected")
    if nodes.dim() != 4 or edges.dim() != 4 or P.dim() != 3 or P.shape[-1] != 2:
        raise _lib.FpmError("feature_align: maps (B, C, H, W) and keypoints (B, nmax, 2) expected")
    B = int(nodes.shape[0])
    nmax = int(P.shape[1]) if nmax is None else int(nmax)
    if int(P.shape[0]) != B or int(P.shape[1]) != nmax or n.numel() != B or n.dtype != torch.int32:
        raise _lib.FpmError("feature_align: P must be (B, nmax, 2) and n (B,) int32")
    P = P.contiguous()
    C = int(nodes.shape[1]) + int(edges.shape[1])
    if out is None:
        out = torch.empty(B * nmax, C, dtype=torch.float32, device=nodes.device)
    if wglob is None:
        wglob = torch.empty(B, int(edges.shape[1]), dtype=torch.float32, device=nodes.device)
    arr = lambda v: ctypes.cast((ctypes.c_long * 4)(*[int(x) for x in v]), ctypes.c_void_p)
    ns_, nst, es_, est = arr(nodes.shape), arr(nodes.stride()), arr(edges.shape), arr(edges.stride())
    lib = _lib.load()
    ws = torch.empty(int(lib.fpm_feature_align_ws_floats(ns_, es_)), dtype=torch.float32, device=nodes.device)
    _lib.call("fpm_feature_align_fwd", _p(nodes), ns_, nst, _p(edges), es_, est, _p(P), _p(n), nmax,
              float(ori_size[0]), float(ori_size[1]), _p(ws), _p(out), int(out.stride(0)), _p(wglob), _stream(nodes))
    return (out, wglob, ws) if keep_ws else (out, wglob)


def feature_align_bwd(nodes, edges, P, n, ws, dX, dwglob=None, ori_size=(320.0, 240.0)):
    """Backward of feature_align: gradients of X rows (and of the global feature) -> gradients of
    the raw maps (dnodes, dedges), allocated with the maps' memory formats."""
    _dev(nodes, edges, P, n, ws, dX)
    B = int(nodes.shape[0])
    nmax = int(P.shape[1])
    Cn, Ce = int(nodes.shape[1]), int(edges.shape[1])
    if dX.dtype != torch.float32 or dX.dim() != 2 or dX.shape[0] != B * nmax or dX.shape[1] < Cn + Ce or dX.stride(1) != 1:
        raise _lib.FpmError("feature_align_bwd: dX must be (B*nmax, >= C_n + C_e) float32 rows")
    if dwglob is not None:
        _shape(dwglob, (B, Ce), "feature_align_bwd dwglob")
        dwglob = dwglob.contiguous().float()
    P = P.contiguous()
    fmt = lambda t: torch.channels_last if t.is_contiguous(memory_format=torch.channels_last) and not t.is_contiguous() \
        else torch.contiguous_format
    dn = torch.empty_like(nodes, memory_format=fmt(nodes))
    de = torch.empty_like(edges, memory_format=fmt(edges))
    arr = lambda v: ctypes.cast((ctypes.c_long * 4)(*[int(x) for x in v]), ctypes.c_void_p)
    _lib.call("fpm_feature_align_bwd", _p(nodes), arr(nodes.shape), arr(nodes.stride()), _p(edges), arr(edges.shape),
              arr(edges.stride()), _p(P), _p(n), nmax, float(ori_size[0]), float(ori_size[1]), _p(ws), _p(dX),
              int(dX.stride(0)), _p(dwglob), _p(dn), arr(dn.stride()), _p(de), arr(de.stride()), _stream(nodes))
    return dn, de


def lsa_batch_device(s, n1, n2, assign=None, status=None):
    """Device LSA (maximise s) over a (B, n1max, n2max) float32 view with unit column stride ->
    (assign (B, n1max) int32, status (B,) int32); bit-identical to ``lsa_batch_host``.  Asynchronous:
    check ``status`` (0 ok, 1 infeasible, 2 NaN/-inf) after synchronising."""
    _dev(s, n1, n2)
    if s.dtype != torch.float32 or s.dim() != 3 or s.stride(2) != 1:
        raise _lib.FpmError("lsa_batch_device: (B, n1max, n2max) float32 with unit column stride expected")
    B, n1max, n2max = s.shape
    if assign is None:
        assign = torch.empty(B, n1max, dtype=torch.int32, device=s.device)
    if status is None:
        status = torch.empty(B, dtype=torch.int32, device=s.device)
    _lib.call("fpm_lsa_batch_device", _p(s), int(s.stride(0)), int(s.stride(1)), _p(n1), _p(n2), B, n1max, n2max,
              _p(assign), _p(status), _stream(s))
    return assign, status


def _assign_out(out, B, n1max):
    if out is None:
        return torch.empty(B, n1max, dtype=torch.int32)
    if out.is_cuda or out.dtype != torch.int32 or tuple(out.shape) != (B, n1max) or not out.is_contiguous():
        raise _lib.FpmError("lsa: out must be a contiguous host (B, n1max) int32 tensor")
    return out


def lsa_batch_host(s_host, n1_host, n2_host, nthreads=1, b0=0, out=None):
    """Host LSA (maximise s) over a pinned/CPU float32 (B, n1max, n2max) tensor -> (B, n1max) int32.
    ``b0``: the batch's first pair index in the caller's batch (error messages report b0 + pair);
    ``out``: optional host (B, n1max) int32 result tensor (pinned: its H2D copy stays asynchronous)."""
    if s_host.is_cuda:
        raise _lib.FpmError("lsa_batch_host expects host memory")
    s_host = s_host.contiguous()
    B, n1max, n2max = s_host.shape
    n1c = n1_host.to(torch.int32).contiguous()
    n2c = n2_host.to(torch.int32).contiguous()
    out = _assign_out(out, B, n1max)
    rc = _lib.load().fpm_lsa_batch_host(_p(s_host), n1max * n2max, n2max, _p(n1c), _p(n2c), B, n1max, _p(out),
                                        int(nthreads))
    if rc != 0:
        raise _lib.FpmError("hungarian: pair %d is infeasible or has NaN/-inf costs" % (b0 + rc - 1))
    return out


class LsaTicket:
    """A batch queued on the host LSA workers (``lsa_submit``); holds its tensors until waited.
    Every ticket must be waited (``lsa_wait``) before its tensors are dropped: the workers read the
    cost rows and write the assignment until then (``lsa_drain`` waits for a set of tickets)."""

    def __init__(self, ticket, keep, out, b0=0):
        self.ticket, self._keep, self.out, self.b0 = ticket, keep, out, b0
        self.seconds = 0.0
        self.waited = False


def lsa_submit(s_host, n1_host, n2_host, nthreads=1, b0=0, out=None):
    """Asynchronous ``lsa_batch_host``: queue the batch on the persistent LSA workers (pairs of
    successive batches are served first-in first-out) and return a ticket for ``lsa_wait``.
    ``b0``: the batch's first pair index in the caller's batch (error messages report b0 + pair)."""
    if s_host.is_cuda:
        raise _lib.FpmError("lsa_submit expects host memory")
    s_host = s_host.contiguous()
    B, n1max, n2max = s_host.shape
    n1c = n1_host.to(torch.int32).contiguous()
    n2c = n2_host.to(torch.int32).contiguous()
    out = _assign_out(out, B, n1max)
    t = _lib.load().fpm_lsa_submit(_p(s_host), n1max * n2max, n2max, _p(n1c), _p(n2c), B, n1max, _p(out),
                                   int(nthreads))
    return LsaTicket(t, (s_host, n1c, n2c), out, b0)


def lsa_wait(tk, block=True):
    """The assignment of a ``lsa_submit`` batch ((B, n1max) int32), or None if ``block`` is False
    and it is still running.  ``tk.seconds``: the batch's span on the workers."""
    sec = ctypes.c_double(0.0)
    rc = _lib.load().fpm_lsa_wait(tk.ticket, 1 if block else 0, ctypes.byref(sec))
    if rc == -2:
        return None
    if rc == -1:
        raise _lib.FpmError("lsa_wait: unknown or already waited ticket")
    tk.waited = True
    tk.seconds = sec.value
    if rc != 0:
        raise _lib.FpmError("hungarian: pair %d is infeasible or has NaN/-inf costs" % (tk.b0 + rc - 1))
    return tk.out


def lsa_drain(tickets):
    """Block until every not-yet-waited ticket's batch is done (results and errors discarded): the
    cleanup path of a forward that stops early, so no worker still reads or writes its buffers."""
    for tk in tickets:
        if not tk.waited:
            try:
                lsa_wait(tk)
            except _lib.FpmError:
                pass


# ---- training backward -----------------------------------------------------
def sinkhorn_bwd(s, dp, ds, n1, n2, iters, tau, dummy_row, ws):
    """d/ds of ``sinkhorn`` given dp = d/d(out); s, dp: strided (B, n1max, n2max) views; ds contiguous."""
    _dev(s, dp, ds, n1, n2, ws)
    B, n1max, n2max = s.shape
    if tuple(dp.shape) != (B, n1max, n2max) or not ds.is_contiguous() or tuple(ds.shape) != (B, n1max, n2max):
        raise _lib.FpmError("sinkhorn_bwd: shape mismatch")
    _lib.call("fpm_sinkhorn_log_bwd", _p(s), s.stride(0), s.stride(1), s.stride(2), _p(dp), dp.stride(0),
              dp.stride(1), dp.stride(2), _p(ds), _p(n1), _p(n2), B, n1max, n2max, int(iters), float(tau),
              int(bool(dummy_row)), _p(ws), ws.numel(), _stream(s))
    return ds


def soft_topk_bwd(ss, n1, n2, k, steps, tau, dds):
    """d/dss of ``soft_topk`` (k and steps as used / returned by the forward) -> (B, n1max, n2max)."""
    _dev(ss, n1, n2, k, steps, dds)
    B, n1max, n2max = ss.shape
    if ss.stride(2) != 1 or dds.stride(2) != 1 or tuple(dds.shape) != (B, n1max, n2max):
        raise _lib.FpmError("soft_topk_bwd: (B, n1max, n2max) views with unit column stride expected")
    lib = _lib.load()
    ws = torch.empty(max(int(lib.fpm_soft_topk_bwd_ws_floats(B, n1max, n2max)), 1), device=ss.device,
                     dtype=torch.float32)
    status = torch.zeros(B, device=ss.device, dtype=torch.int32)
    dss = torch.empty(B, n1max, n2max, device=ss.device, dtype=torch.float32)
    _lib.call("fpm_soft_topk_bwd", _p(ss), ss.stride(0), ss.stride(1), _p(n1), _p(n2), _p(k), _p(steps), B, n1max,
              n2max, float(tau), _p(dds), dds.stride(0), dds.stride(1), _p(dss), _p(ws), ws.numel(), _p(status),
              _stream(ss))
    if int(status.sum()):
        raise _lib.FpmError("soft_topk_bwd: forward ran more steps than the backward replay holds")
    return dss


def spline_plan_rows(plan, E, num_nodes):
    """(arows, cell_off) int32 views into a plan: product row -> source node, per-cell row ranges."""
    a, c = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.call("fpm_spline_plan_rows", _p(plan), E, num_nodes, ctypes.byref(a), ctypes.byref(c))
    base = plan.data_ptr()
    oa, oc = a.value - base, c.value - base
    arows = plan[oa:].view(torch.int32)
    cell_off = plan[oc:oc + 4 * 27].view(torch.int32)
    return arows, cell_off


def spline_conv_bwd_data(x_op, plan, E, num_nodes, nmax, nvalid, Wb, y_ws, mode, gout, hout, dY, dY_op, dXrows, dX,
                         accumulate=False, rplan=None, argmax=None):
    """Input gradient of one SplineConv layer (see include/fpm.h); fills dY (product-row grads).
    rplan (plan of the reversed edges) + argmax (from spline_conv(..., argmax=)): the atomic-free
    scatter form."""
    _dev(plan, nvalid, Wb, y_ws, gout, dY, dXrows, dX)
    code = _code(x_op)
    if _code(Wb) != code or tuple(Wb.shape) != (26, 768, 768):
        raise _lib.FpmError("spline_conv_bwd: Wb must be (26, 768, 768) in the operand dtype")
    if mode == 0 and hout is None:
        raise _lib.FpmError("spline_conv_bwd: mode 0 needs the layer output")
    if (rplan is None) != (argmax is None):
        raise _lib.FpmError("spline_conv_bwd: rplan and argmax go together")
    _lib.call("fpm_spline_conv_bwd_data_scatter", code, _p(plan), _p(rplan), _p(argmax), E, num_nodes, nmax,
              _p(nvalid), _p(Wb), _p(y_ws), int(mode), _p(gout), _p(hout), _p(dY), _p(dY_op), _p(dXrows), _p(dX),
              int(bool(accumulate)), _stream(gout))


def kron_agg(X, C, B, n1max, n2max, tcsr1, tcsr2, q1, q2, n1, n2, adjoint, out, accumulate=False):
    """Factorised Kronecker SAGE-mean aggregation (adjoint=False: forward agg over the in-edge CSRs
    tcsr*; adjoint=True: its transpose over the out-edge CSRs).  q1/q2: in-edge CSR pointers.
    ``accumulate``: out += result."""
    _dev(X, n1, n2, out)
    _lib.call("fpm_kron_agg", _p(X), int(C), int(B), int(n1max), int(n2max), ctypes.c_void_p(tcsr1[0]),
              ctypes.c_void_p(tcsr1[1]), ctypes.c_void_p(tcsr2[0]), ctypes.c_void_p(tcsr2[1]), ctypes.c_void_p(q1),
              ctypes.c_void_p(q2), _p(n1), _p(n2), int(bool(adjoint)) | (2 if accumulate else 0), _p(out), _stream(X))
    return out


def gnn_layer_bwd_point(X, C, B, n1max, n2max, dXn, dz, params, dX, dagg, V):
    """Per-position PYGNNLayer backward (node MLPs + classifier): dX (direct part), dagg, and
    V = [dx1 | dh1 | dm | h1] (B, 64, N) for the weight-gradient reductions."""
    _dev(X, dXn, dz, params, dX, dagg, V)
    for t in (X, dXn, dz, dX, dagg, V):
        if not t.is_contiguous():
            raise _lib.FpmError("gnn_layer_bwd_point: contiguous tensors expected")
    _lib.call("fpm_kron_gnn_layer_bwd_point", _p(X), int(C), int(B), int(n1max), int(n2max), _p(dXn), _p(dz),
              _p(params), _p(dX), _p(dagg), _p(V), _stream(X))


def _counts(n, B, full, dev):
    """nrows / ncols as the kernels take them: int32 on ``dev``; None -> the unpadded size."""
    if n is None:
        return torch.full((B,), int(full), dtype=torch.int32, device=dev)
    return torch.as_tensor(n).reshape(-1).to(device=dev, dtype=torch.int32)


class Sinkhorn(torch.nn.Module):
    """``Sinkhorn(max_iter=10, tau=1., epsilon=1e-4, log_forward=True, batched_operation=False)``
    (``src/model/sinkhorn.py:7-87``), whose ``forward_log`` is ``pygmtools.sinkhorn``: log-domain
    alternating row / column normalisation of ``s / tau`` on each pair's valid block, dummy rows
    when asked, pairs with n1 > n2 run transposed.  Differentiable (``fpm_sinkhorn_log_bwd``).
    ``epsilon`` and ``batched_operation`` do not change the log-domain result and are accepted
    for signature parity."""

    def __init__(self, max_iter=10, tau=1., epsilon=1e-4, log_forward=True, batched_operation=False):
        super().__init__()
        if not log_forward:
            # forward_ori is deprecated in the reference (sinkhorn.py:53-54); only the log form is built
            raise NotImplementedError("Sinkhorn(log_forward=False) is not built: use the log-domain forward")
        self.max_iter, self.tau, self.epsilon = max_iter, tau, epsilon
        self.log_forward, self.batched_operation = log_forward, batched_operation

    def forward(self, s, nrows=None, ncols=None, dummy_row=False):
        return self.forward_log(s, nrows, ncols, dummy_row)

    def forward_log(self, s, nrows=None, ncols=None, dummy_row=False):
        _dev(s)
        matrix_input = s.dim() == 2
        if matrix_input:
            s = s.unsqueeze(0)
        if s.dim() != 3:
            raise ValueError("input data shape not understood: %s" % (tuple(s.shape),))
        B, n1max, n2max = s.shape
        n1 = _counts(nrows, B, n1max, s.device)
        n2 = _counts(ncols, B, n2max, s.device)
        sf = s.float()
        if sf.requires_grad and torch.is_grad_enabled():
            from .train import SinkhornFn
            out = SinkhornFn.apply(sf, n1, n2, int(self.max_iter), float(self.tau), bool(dummy_row))
        else:
            out = sinkhorn(sf.detach(), n1, n2, int(self.max_iter), float(self.tau), bool(dummy_row))
        out = out.to(s.dtype)
        return out.squeeze(0) if matrix_input else out


def greedy_perm(x, top_indices, ks):
    """``greedy_perm(x, top_indices, ks)`` (``src/model/soft_topk.py:56-77``): walk each pair's
    candidate order and accept (idx // n2max, idx % n2max) while its row and column of ``x`` still
    sum to < 1, until ``round(ks[b])`` (half-to-even) are accepted.  ``x`` is updated in place and
    returned (fpm_greedy_perm)."""
    _dev(x, top_indices)
    if x.dim() != 3 or x.dtype != torch.float32 or x.stride(2) != 1:
        raise _lib.FpmError("greedy_perm: x must be a (b, n1, n2) float32 tensor with unit column stride")
    B, n1max, n2max = x.shape
    top = top_indices.reshape(B, -1).to(torch.int64).contiguous()
    k = torch.as_tensor(ks).reshape(-1).to(device=x.device, dtype=torch.float32).contiguous()
    if k.numel() != B:
        raise _lib.FpmError("greedy_perm: ks must hold one count per pair")
    _lib.call("fpm_greedy_perm", _p(top), top.stride(0), int(top.shape[1]), _p(k), B, n1max, n2max, _p(x),
              x.stride(0), x.stride(1), _stream(x))
    return x


def soft_topk(scores, ks, max_iter=10, tau=1., nrows=None, ncols=None, return_prob=False):
    """``soft_topk(scores, ks, max_iter, tau, nrows, ncols, return_prob)``
    (``src/model/soft_topk.py:8-53``): the 2-column marginal Sinkhorn incl. ``Sinkhorn_m``'s
    data-dependent continuation (fpm_soft_topk_fwd), then the reference's own hard output:
    candidates in descending order of P(top-k) over the pair's flattened valid block
    (q = i * n2 + j, padded to max(nrows) * max(ncols) with zeros), decoded with the box width
    like the reference's greedy_perm.  Ties keep ascending flat index (the reference's argsort is
    unstable, quirk A.10(v)).  Returns x, or (x, soft matrix) with ``return_prob``.  The soft
    matrix is differentiable in ``scores`` (fpm_soft_topk_bwd)."""
    _dev(scores)
    B, n1max, n2max = scores.shape
    n1 = _counts(nrows, B, n1max, scores.device)
    n2 = _counts(ncols, B, n2max, scores.device)
    k = torch.as_tensor(ks).reshape(-1).to(device=scores.device, dtype=torch.float32)
    sf = scores.float()
    if sf.requires_grad and torch.is_grad_enabled():
        from .train import SoftTopkFn
        out_s = SoftTopkFn.apply(sf, k, n1, n2, int(max_iter), float(tau))
    else:
        out_s = soft_topk_fwd(sf.detach().contiguous(), n1, n2, k.contiguous(), int(max_iter), float(tau))
    # the reference's output[:, :, 1]: (b, max(nrows) * max(ncols)), pair b's block row-major first
    L = int(n1.max()) * int(n2.max())
    q = torch.arange(L, device=scores.device)
    n2l = n2.long()[:, None]
    valid = q[None, :] < (n1.long() * n2.long())[:, None]
    flat = out_s.detach()[torch.arange(B, device=scores.device)[:, None],
                          torch.where(valid, q[None, :] // n2l, 0), torch.where(valid, q[None, :] % n2l, 0)]
    flat = torch.where(valid, flat, torch.zeros((), device=scores.device))
    top = torch.argsort(flat, dim=-1, descending=True, stable=True)
    x = greedy_perm(torch.zeros(B, n1max, n2max, device=scores.device), top, k)
    x = x.to(scores.dtype)
    return (x, out_s.to(scores.dtype)) if return_prob else x


def hungarian(s, n1=None, n2=None, nproc=1):
    """``hungarian(s, n1, n2, nproc)`` (``utils/hungarian.py:8-66``): the optimal assignment
    maximising ``s`` on each pair's valid block (scipy ``linear_sum_assignment`` of ``-s``, same
    tie rules) -> 0/1 matrix of ``s``'s shape, dtype and device.  Solved on the host LSA pool
    (fpm_lsa_batch_host, ``nproc`` threads) as the reference solves it on the host."""
    matrix_input = s.dim() == 2
    if matrix_input:
        s = s.unsqueeze(0)
    elif s.dim() != 3:
        raise ValueError("input data shape not understood: %s" % (tuple(s.shape),))
    B, n1max, n2max = s.shape
    host = s.detach().to("cpu", torch.float32).contiguous()
    a = lsa_batch_host(host, _counts(n1, B, n1max, "cpu"), _counts(n2, B, n2max, "cpu"), max(1, int(nproc)))
    perm = torch.zeros(B, n1max, n2max, dtype=torch.float32)
    r = torch.nonzero(a >= 0)
    perm[r[:, 0], r[:, 1], a[r[:, 0], r[:, 1]].long()] = 1.0
    perm = perm.to(device=s.device, dtype=s.dtype)
    return perm.squeeze(0) if matrix_input else perm


