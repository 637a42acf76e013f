"""ctypes binding of ``libfpm_hip.so`` (C-ABI declared in ``include/fpm.h``).

The library is loaded from this package directory (built in-tree by ``build.py``).  There is no
fallback: if the library is missing every op raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FPM_LIB_PATH: an alternative in-tree build (A/B timing of two builds in one GPU call)
LIB_PATH = os.environ.get("FPM_LIB_PATH") or os.path.join(_HERE, "libfpm_hip.so")

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float

# name -> (restype, argtypes)
SIGNATURES = {
    "fpm_last_error": (ctypes.c_char_p, []),
    "fpm_version": (I, []),
    "fpm_device_sync": (I, []),
    "fpm_sinkhorn_log_fwd": (I, [P, L, L, L, P, L, L, L, P, P, I, I, I, I, F, I, P]),
    "fpm_sinkhorn_ws_bytes": (L, [I, I, I]),
    "fpm_sinkhorn_log_fwd_ws": (I, [P, L, L, L, P, L, L, L, P, P, I, I, I, I, F, I, P, L, P]),
    "fpm_soft_topk_fwd": (I, [P, L, L, P, P, P, I, I, I, I, F, P, L, L, P, P, L, L, P]),
    "fpm_topk_select": (I, [P, L, L, P, L, P, I, I, I, P, L, L, P, L, L, P]),
    "fpm_greedy_perm": (I, [P, L, I, P, I, I, I, P, L, L, P]),
    "fpm_gemm": (I, [I, P, L, L, P, P, L, L, I, I, I, I, I, P, P, P, L, L, P, P, P]),
    "fpm_cast_bf16": (I, [P, P, L, P]),
    "fpm_global_weights": (I, [P, L, P, L, I, I, I, P, L, P]),
    "fpm_coef_tanh": (I, [P, L, P, P, I, I, I, P, L, P]),
    "fpm_split_bf16x3": (I, [P, L, L, I, I, P, L, P]),
    "fpm_set_tuning": (I, [ctypes.c_char_p, I]),
    "fpm_spline_plan_bytes": (L, [L, L]),
    "fpm_spline_plan": (I, [P, P, P, L, L, I, P, L, P]),
    "fpm_spline_plan_graphs": (I, [P, P, P, L, L, I, L, P, L, P]),
    "fpm_spline_plan_csr": (I, [P, L, L, ctypes.POINTER(P), ctypes.POINTER(P)]),
    "fpm_spline_plan_multi": (I, [P, I, I, I, P, P]),
    "fpm_spline_plan_job_bytes": (I, []),
    "fpm_spline_y_bytes": (L, [I, L, L]),
    "fpm_spline_conv_fwd": (I, [I, P, P, L, L, I, P, P, P, P, L, I, P, P, P, P, P]),
    "fpm_spline_conv_fwd_argmax": (I, [I, P, P, L, L, I, P, P, P, P, L, I, P, P, P, P, P, P]),
    "fpm_edge_diff": (I, [P, P, P, L, I, P, P]),
    "fpm_rows_bcast_scale": (I, [I, P, L, I, P, P, P, I, P]),
    "fpm_edge_diff_padded": (I, [P, P, P, P, P, P, L, I, P, P]),
    "fpm_kron_gnn_layer_fwd": (I, [P, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P]),
    "fpm_kron_gnn_layer_fwd_ord": (I, [P, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "fpm_gnn_param_count": (I, [I]),
    "fpm_node_classifier": (I, [P, I, I, I, P, P, P, P, P]),
    "fpm_crossset_attn_fwd": (I, [I, P, L, L, I, I, I, P, P, I, P, P, P, P, P, P, P]),
    "fpm_instnorm": (I, [I, P, P, I, I, I, P, P, P, P, F, P, P, I, P, P]),
    "fpm_afau_head": (I, [P, P, I, I, P, P, P, P, P, P, P, P, P, P]),
    "fpm_afau_head_bwd": (I, [P, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "fpm_instnorm_bwd": (I, [P, P, I, I, I, P, P, P, P, F, P, P, P, I, P, P, P]),
    "fpm_afau_attn_bwd": (I, [P, L, L, I, I, I, P, P, I, P, P, P, P, P, P, P, P, P, P]),
    "fpm_rows_sum": (I, [P, I, L, P, I, P, I, P]),
    "fpm_transpose": (I, [P, L, I, L, P, L, P]),
    "fpm_elementwise": (I, [P, P, L, I, P]),
    "fpm_outer_sum_parts": (L, [I, L]),
    "fpm_outer_sum": (I, [P, L, L, I, P, L, L, I, I, I, L, P, P]),
    "fpm_bn_ws_floats": (L, [I, I]),
    "fpm_bn_relu_train_fwd": (I, [P, I, I, L, P, P, F, F, P, P, P, P, P, P]),
    "fpm_bn_relu_train_bwd": (I, [P, P, I, I, L, P, P, P, P, P, P, P]),
    "fpm_match_cls_ws_floats": (L, [I, I, I]),
    "fpm_match_cls_fwd": (I, [I, P, P, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "fpm_match_cls_train_ws_floats": (L, [I, I, I, I]),
    "fpm_match_cls_train_fwd": (I, [P, P, I, I, I] + [P] * 14 + [ctypes.c_float, ctypes.c_float, P, P, P, P]),
    "fpm_match_cls_train_bwd": (I, [P, P, I, I, I] + [P] * 21 + [P]),
    "fpm_gemm_norm_max": (I, [P, L, P, L, I, I, I, P, P, L, P, P, ctypes.c_float, I, P, P]),
    "fpm_gemm_norm_out": (I, [P, L, P, L, I, I, I, P, P, P, ctypes.c_float, I, P, L, P, L, P]),
    "fpm_affinity_ws_floats": (L, [I, I, I]),
    "fpm_perm_loss_fwd": (I, [P, L, L, P, L, L, P, P, I, I, I, P, P, P, P]),
    "fpm_perm_loss_bwd": (I, [P, L, L, P, L, L, P, P, I, I, I, P, P, P, P]),
    "fpm_affinity_fwd": (I, [P, L, P, L, P, I, P, P, I, I, I, I, P, P, I, P, L, P, L, P]),
    "fpm_gemm_x3out": (I, [P, L, P, L, I, I, I, I, P, P, P, ctypes.c_float, I, P, L, P, L, I, P]),
    "fpm_lsa_batch_host": (I, [P, L, L, P, P, I, I, P, I]),
    "fpm_lsa_submit": (L, [P, L, L, P, P, I, I, P, I]),
    "fpm_lsa_wait": (I, [L, I, ctypes.POINTER(ctypes.c_double)]),
    "fpm_lsa_batch_device": (I, [P, L, L, P, P, I, I, I, P, P, P]),
    "fpm_csr_dot_csc_to_dense": (I, [I, P, P, P, P, P, P, L, L, L, P, P]),
    "fpm_dense_dot_csc_to_dense": (I, [I, P, P, P, P, L, L, L, L, P, P]),
    "fpm_csr_dot_diag_to_csr": (I, [I, P, P, P, P, L, L, L, P, P]),
    "fpm_bilinear_diag": (I, [I, P, P, P, P, L, P, P, P, L, L, P, P]),
    "fpm_csr_dot_csc_to_csr_host": (L, [I, P, P, P, P, P, P, L, L, L, P, L, P, P]),
    "fpm_csr_dot_diag_to_csr_host": (I, [I, P, P, P, P, L, L, L, P]),
    "fpm_bilinear_diag_host": (I, [I, P, P, P, P, L, P, P, P, L, L, P]),
    "fpm_gconv_ws_floats": (L, [I, I, I]),
    "fpm_gconv_fwd": (I, [P, P, I, I, I, I, P, P, I, P, P, P]),
    "fpm_graph_words": (I, [I]),
    "fpm_graph_build": (I, [P, P, I, I, I, ctypes.c_double, P, P, P, P, P]),
    "fpm_graph_edges": (I, [P, P, P, P, I, I, ctypes.c_double, P, P, P, P, P, P, I, P]),
    "fpm_kron_pattern": (I, [P, P, L, P, P, L, I, I, I, I, P, P, P]),
    "fpm_feature_align_ws_floats": (L, [P, P]),
    "fpm_feature_align_fwd": (I, [P, P, P, P, P, P, P, P, I, F, F, P, P, L, P, P]),
    "fpm_feature_align_bwd": (I, [P, P, P, P, P, P, P, P, I, F, F, P, P, L, P, P, P, P, P, P]),
    "fpm_sinkhorn_bwd_ws_floats": (L, [I, I, I, I]),
    "fpm_sinkhorn_log_bwd": (I, [P, L, L, L, P, L, L, L, P, P, P, I, I, I, I, F, I, P, L, P]),
    "fpm_soft_topk_bwd_ws_floats": (L, [I, I, I]),
    "fpm_soft_topk_bwd": (I, [P, L, L, P, P, P, P, I, I, I, F, P, L, L, P, P, L, P, P]),
    "fpm_spline_plan_rows": (I, [P, L, L, ctypes.POINTER(P), ctypes.POINTER(P)]),
    "fpm_spline_conv_bwd_data": (I, [I, P, L, L, I, P, P, P, I, P, P, P, P, P, P, I, P]),
    "fpm_gather_transpose": (I, [I, P, L, P, L, I, P, L, P]),
    "fpm_spline_weight_pack": (I, [P, P, I, I, I, I, I, P, P]),
    "fpm_spline_conv_bwd_data_scatter": (I, [I, P, P, P, L, L, I, P, P, P, I, P, P, P, P, P, P, I, P]),
    "fpm_kron_agg": (I, [P, I, I, I, I, P, P, P, P, P, P, P, P, I, P, P]),
    "fpm_kron_gnn_layer_bwd_point": (I, [P, I, I, I, I, P, P, P, P, P, P, P]),
    "fpm_kron_gnn_layer_fwd_f64": (I, [P, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P]),
    "fpm_sinkhorn_log_fwd_f64": (I, [P, I, L, L, L, P, L, L, L, P, L, L, L, P, P, I, I, I, I, ctypes.c_double, I, P]),
    "fpm_node_classifier_f64": (I, [P, I, I, I, P, P, P, P, P]),
    "fpm_crossset_attn_row_f64": (I, [P, L, L, I, I, I, P, P, I, P, P, P, P, P, P]),
    "fpm_gemm_f64": (I, [P, I, P, I, P, P, I, I, I, I, I, P]),
    "fpm_instnorm_f64": (I, [P, P, I, I, I, P, P, P, P, ctypes.c_double, P, P, P]),
    "fpm_afau_head_f64": (I, [P, P, P, I, I, P, P, P, P, P, P, P, P, P, P]),
    "fpm_soft_topk_fwd_f64": (I, [P, L, L, P, P, P, I, I, I, I, ctypes.c_double, P, L, P, L, L, P, P, L, L, P]),
    "fpm_profile_enable": (I, [I]),
    "fpm_profile_enabled": (I, []),
    "fpm_profile_read": (I, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(I)]),
}

_lib = None


class FpmError(RuntimeError):
    pass


def load():
    """Load the HIP library once; raise loudly if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FpmError("libfpm_hip.so not found at %s — build it with "
                       "`python fingerprint-matching-code_amd/build.py` (no CPU fallback exists)" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def call(name, *args):
    """Invoke a status-returning C-ABI function; raise FpmError with fpm_last_error() on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.fpm_last_error().decode(errors="replace")
        raise FpmError("%s failed (status %d): %s" % (name, rc, msg))
    return rc
