/*
 * fpm.h — C-ABI of libfpm_hip.so, the MI355X (gfx950) graph-matching forward of the fingerprint
 * QAP matcher (reference: dayne-2stacks/Fingerprint-Matching-Code).
 *
 * Conventions
 *   - extern "C", plain pointers and sizes; no C++/torch types cross the boundary.
 *   - Return value: 0 = ok, nonzero = error; fpm_last_error() returns a thread-local message.
 *   - Device ops take a hipStream_t (passed as void*) and are asynchronous on it.
 *   - The caller allocates every output and workspace (device memory unless noted "host").
 *   - dtype codes for MFMA operands: 0 = fp32, 1 = bf16 (raw 16-bit); accumulation is fp32.
 *   - Batched matrices are addressed by (base, batch stride, row stride[, col stride]) in elements.
 *
 * What this replaces: the reference's pybind11 extensions JIT-built at import time
 * (src/sparse_torch/csx_matrix.py:10-17, src/sparse.py:12-16) and the third-party operators its
 * live forward calls (PyG SplineConv/SAGEConv, torch_sparse, pygmtools, scipy LSA).  Each entry
 * point cites the reference interface it stands in for.
 */
#ifndef FPM_H_
#define FPM_H_

#ifdef __cplusplus
extern "C" {
#endif

/* ---- plumbing ------------------------------------------------------------------------------ */
const char* fpm_last_error(void);
int fpm_version(void);
int fpm_device_sync(void);

/* ---- log-domain Sinkhorn ---------------------------------------------------------------------
 * Replaces Sinkhorn.forward_log -> pygmtools.sinkhorn (src/model/sinkhorn.py:85-87), used by
 * PYGNNLayer (src/model/gnn.py:221, 20 iterations) and Net.forward (ngm.py:371, 10 iterations).
 * out[b] = exp(L) on the valid block [:n1[b], :n2[b]] of the (n1max, n2max) box, 0 elsewhere.
 * Any strides.  n1max, n2max <= 256 run VGPR-resident (one workgroup per pair); larger boxes, up
 * to 2048, stream the block through L2 (same arithmetic, fpm_sinkhorn_log_fwd picks the variant). */
int fpm_sinkhorn_log_fwd(const float* s, long s_sb, long s_si, long s_sj, float* out, long o_sb, long o_si,
                         long o_sj, const int* n1, const int* n2, int B, int n1max, int n2max, int iters,
                         float tau, int dummy_row, void* stream);
/* The same with a caller-provided device workspace of fpm_sinkhorn_ws_bytes(B, n1max, n2max) bytes
 * (16-B aligned; 0 = none needed): boxes over 256 then run each pair on FPM_SK_SPLIT (default 2)
 * workgroups that exchange their partial column sums through it, instead of one workgroup per pair
 * (fp32 summation order of the column sums differs; both forms within the oracle's tolerance).
 * Concurrent calls need separate workspaces. */
long fpm_sinkhorn_ws_bytes(int B, int n1max, int n2max);
int fpm_sinkhorn_log_fwd_ws(const float* s, long s_sb, long s_si, long s_sj, float* out, long o_sb, long o_si,
                            long o_sj, const int* n1, const int* n2, int B, int n1max, int n2max, int iters,
                            float tau, int dummy_row, void* ws, long ws_bytes, void* stream);

/* ---- soft top-k -------------------------------------------------------------------------------
 * Replaces soft_topk(..., return_prob=True)[1] (src/model/soft_topk.py:8-53) incl. Sinkhorn_m's
 * data-dependent continuation (:232-241).  k[b] = number of matches (ks * min(n1,n2) in eval).
 * steps_out (optional, int32[B]) receives the number of normalisation steps run. */
int fpm_soft_topk_fwd(const float* ss, long s_sb, long s_ld, const int* n1, const int* n2, const float* k, int B,
                      int n1max, int n2max, int iters, float tau, float* out, long o_sb, long o_ld, int* steps_out,
                      float* out2, long o2_sb, long o2_ld, void* stream);

/* ---- greedy top-k selection -------------------------------------------------------------------
 * Replaces argsort(x * ss_out) + greedy_perm (ngm.py:445-449, soft_topk.py:56-77).  n1max, n2max <= 2048.
 * assign[b][r] = column matched to row r by the LSA (or -1); perm receives the 0/1 matrix;
 * lsa_out (optional) receives the dense LSA matrix x. */
int fpm_topk_select(const float* ds, long d_sb, long d_ld, const int* assign, long a_sb, const float* k, int B,
                    int n1max, int n2max, float* perm, long p_sb, long p_ld, float* lsa_out, long l_sb, long l_ld,
                    void* stream);

/* ---- greedy_perm for an arbitrary candidate order ---------------------------------------------
 * Replaces greedy_perm(x, top_indices, ks) (src/model/soft_topk.py:56-77) as called inside
 * soft_topk (:40-41).  top_idx[b][0..T) (int64, flat indices into the (n1max, n2max) box, decoded
 * as idx / n2max, idx % n2max like the reference); x is updated in place (rows / columns whose sum
 * is >= 1 are taken).  k[b] is rounded half-to-even.  n1max, n2max <= 2048. */
int fpm_greedy_perm(const long* top_idx, long t_sb, int T, const float* k, int B, int n1max, int n2max, float* x,
                    long x_sb, long x_ld, void* stream);

/* ---- global weights ---------------------------------------------------------------------------
 * Replaces normalize_over_channels(cat(global_src, global_tgt)) (src/model/ngm.py:65-67, 262-268):
 * out[b] = cat(w1[b], w2[b]) / ||cat(w1[b], w2[b])||_2, reduced in a fixed per-pair order. */
int fpm_global_weights(const float* w1, long ld1, const float* w2, long ld2, int B, int D1, int D2, float* out,
                       long ldo, void* stream);

/* ---- split-bf16 operands ------------------------------------------------------------------------
 * dst[r] = [hi | lo | hi] (bf16, each Kp wide, zero-padded from K), hi = bf16(src[r]),
 * lo = bf16(src[r] - hi): the A operand of a near-fp32 product on the bf16 MFMA path (weights
 * packed [B_hi | B_hi | B_lo]); used for the AFA-U projections (afau.py:99-103, 188-199). */
int fpm_split_bf16x3(const float* src, long lds, long rows, int K, int Kp, void* dst, long ldd, void* stream);

/* ---- generic MFMA GEMM with fused epilogue ----------------------------------------------------
 * C[b][r][n] = epi(sum_k A[b][row(r)][k] * B[b][n][k] (+ bias[n])), row(r) = a_rows ? a_rows[r] : r.
 * epi: 0 store, 1 relu, 2 tanh, 3 affinity (softplus(v) - 0.5 inside [:n2[b], :n1[b]], else 0).
 * Stands in for nn.Linear / torch.matmul on the hot path: InnerProductWithWeightsAffinity
 * (affinity_layer.py:13-18), AFA-U projections and FFN (afau.py:99-103, 188-199). */
int fpm_gemm(int dtype, const void* A, long lda, long sA, const int* a_rows, const void* B, long ldb, long sB, int M,
             int N, int K, int batch, int epi, const float* bias, float* Cf, void* Ct, long ldc, long sC,
             const int* n1, const int* n2, void* stream);
int fpm_cast_bf16(const float* x, void* y, long n, void* stream);
/* AFA-U encoder block tail fused into the FFN's second GEMM (afau.py:188-199 InstanceNorm1d, then
 * the max over positions taken by the caller, afau.py:231-300): per pair b (P = 256 rows, one GEMM
 * tile) gmax[b][n] = max_p ((v - mean_p v) / sqrt(var_p v + eps) * nw[n] + nb[n]),
 * v = res[b P + p][n] + (A B^T)[b P + p][n] + bias[n]; bf16 A (M x K, lda) and B (N x K, ldb). */
int fpm_gemm_norm_max(const void* A, long lda, const void* B, long ldb, int M, int N, int K, const float* bias,
                      const float* res, long ldres, const float* nw, const float* nb, float eps, int P, float* gmax,
                      void* stream);
/* AFA-U encoder block head (afau.py:188-199, the first InstanceNorm1d on the attention-combine
 * projection afau.py:231-300): out_f[b P + p][n] = ((v - mean_p v) / sqrt(var_p v + eps)) * nw[n] +
 * nb[n], v = (A B^T)[b P + p][n] + bias[n], P = 256 rows per pair (one GEMM tile); out_t (optional)
 * its bf16 copy, row stride ldt, columns [N, ldt) written as zeros (the next GEMM's K padding). */
int fpm_gemm_norm_out(const void* A, long lda, const void* B, long ldb, int M, int N, int K, const float* bias,
                      const float* nw, const float* nb, float eps, int P, float* out_f, long ldc, void* out_t, long ldt,
                      void* stream);
/* ---- affinity (the surveyed entry point) -------------------------------------------
 * Replaces InnerProductWithWeightsAffinity._forward (src/model/affinity_layer.py:11-19) for a batch
 * of pairs: c[b] = tanh(A_w w[b] + A_b); K[b][i][j] = epi(((X1[b] o c[b]) X2[b]^T)[i][j]) for
 * i < n1[b], j < n2[b], else 0; epi 0 = softplus(v) - 0.5 (vertex affinity, ngm.py:277-280),
 * 1 = 0.5 (softplus(v) - 0.5) (edge affinity Ke, ngm.py:282-287).  fp32 operands and arithmetic (the
 * fp32 MFMA GEMM).  X1: (B n1max, d) rows (stride ld1), X2: (B n2max, d) (stride ld2), w: (B, kw),
 * A_w: (d, kw), K: (B, n1max, n2max) with row stride ldk (batch stride n1max ldk).  ws: caller
 * workspace of fpm_affinity_ws_floats(B, n1max, d) floats.  (Net's forward fuses the same steps:
 * the coefficients in one tanh GEMM per forward, X1 o c in the SplineConv epilogue, Kp^T in the
 * GNN's layout by a bf16 / fp32 GEMM with this epilogue.) */
/* the forward's affinity coefficients c[b][n] = tanh(sum_k g[b][k] wT[k][n] + bias[n]) (the global-weight
 * projection of InnerProductWithWeightsAffinity, affinity_layer.py:13), wT the [K][N] transposed
 * weight, K <= 1024; each output's fp32 sum = four ascending-k partial chains over the K quarters, added
 * in quarter order -- the same whatever B is */
int fpm_coef_tanh(const float* g, long ldg, const float* wT, const float* bias, int B, int K, int N, float* out,
                  long ldo, void* stream);
long fpm_affinity_ws_floats(int B, int n1max, int d);
int fpm_affinity_fwd(const float* X1, long ld1, const float* X2, long ld2, const float* w, int kw, const float* A_w,
                     const float* A_b, int B, int n1max, int n2max, int d, const int* n1, const int* n2, int epi,
                     float* K, long ldk, float* ws, long ws_floats, void* stream);

/* ---- PermutationLoss (src/loss_func.py:26-59), training ------------------------------------------
 * out[0] = sum_b sum_{i < n1[b], j < n2[b]} BCE(ds[b][i][j], gt[b][i][j]) / sum_b n1[b] with torch's
 * clamped logs (max(log, -100)); pairs summed in a fixed order (one workgroup per pair, then the pair
 * partials in order).  ws: B floats.  The backward writes dds (contiguous B x n1max x n2max) =
 * g[0] (x - t) / max((1 - x) x, 1e-12) / sum n1 on the valid blocks, 0 elsewhere (g, ws: one
 * float each, device).  n1[b] / n2[b] are clamped to the padded box n1max x n2max (the reference's
 * slice ds[b, :n1, :n2] clamps the same way); bad (optional, B ints, device): bad[b] = 1 iff pair b's
 * block holds a ds or gt entry outside [0, 1] or NaN -- the reference's range assert
 * (loss_func.py:42-47), checked by the caller. */
int fpm_perm_loss_fwd(const float* ds, long d_sb, long d_ld, const float* gt, long g_sb, long g_ld, const int* n1,
                      const int* n2, int B, int n1max, int n2max, float* ws, int* bad, float* out, void* stream);
int fpm_perm_loss_bwd(const float* ds, long d_sb, long d_ld, const float* gt, long g_sb, long g_ld, const int* n1,
                      const int* n2, int B, int n1max, int n2max, const float* g, float* ws, float* dds, void* stream);

/* Near-fp32 operands straight from a GEMM epilogue (the gate-passing bf16x3 AFA-U mode,
 * afau.py:99-103, 188-199): C = epi(A B^T + bias) in fp32 on the bf16 MFMA path, written as split
 * rows out_t3[r] = [hi | lo | hi] (segment stride Kp, columns [N, Kp) of each segment zero, row
 * stride ldt >= 3 Kp; identical to fpm_split_bf16x3 of the fp32 result) and, if out_f is non-null,
 * as fp32 rows (stride ldc).  epi: 0 store, 1 relu, 6 (EPI_NORM_OUT) InstanceNorm over each pair's
 * P = 256 rows with weights nw / nb (out_f required), as fpm_gemm_norm_out. */
int fpm_gemm_x3out(const void* A, long lda, const void* B, long ldb, int M, int N, int K, int epi, const float* bias,
                   const float* nw, const float* nb, float eps, int P, float* out_f, long ldc, void* out_t3, long ldt,
                   int Kp, void* stream);
/* Kernel-variant switches for A/B timing.  Returns the
 * previous value, or -1 (error channel set) for an unknown key.  No reference counterpart.
 *   "gemm_phase" (env FPM_GEMM_PHASE, default 1): 256x256 bf16 GEMM tiles on the phase-pipelined
 *                kernel (1) or the two-stage kernel (0)
 *   "combine_npb" (FPM_COMBINE_NPB, default 4): destination nodes per SplineConv combine workgroup
 *   "plan_graph" (FPM_PLAN_GRAPH, default 1): per-graph spline plan kernels where they apply (1) or
 *                the global plan kernels (0)
 *   "sinkhorn_bwd_reg" (FPM_SINKHORN_BWD_REG, default 1): register-tile Sinkhorn backward (n <= 256)
 *   "afau_attn_v" (default 1): the LDS-staged-V cross-set attention where it applies (n2max <= 512)
 *   "gnn_store_sc1" (FPM_GNN_SC1), "combine_store_sc1" (FPM_COMBINE_SC1), "gemm_store_sc1"
 *                (FPM_GEMM_SC1), default 0: the GNN layer's / SplineConv combine's / product GEMM's output
 *                stores with the sc1 cache policy (the lines leave the XCD's L2); same bytes
 *   "combine_lds_kb" (default 0): dynamic LDS reserved per combine workgroup (a residency cap)
 *   "gnn_mlp_off" (default 0): timing probe only -- the GNN layer without its node MLPs (wrong results);
 *                refused (-1) unless the environment has FPM_TIMING_PROBES=1, and fpm.Net refuses to run
 *                while it is set
 *   "outer_sum_vec" (default 1): fpm_outer_sum stages 16-B row pieces when every row start is
 *                16-B aligned (0: one 4-B load per row and position); same products, same order
 *   "gnn_sweeps" (FPM_GNN_SWEEPS, default 1): the 17-channel GNN layer's graph-2 neighbour rows
 *                read in 1 / 2 / 3 channel-group sweeps (same sums, same order; 2 and 3 measured slower)
 *   "scatter_f32_rows" (FPM_SCATTER_F32_ROWS, default 0): the bf16 scatter SplineConv backward also
 *                writes its fp32 cell rows of dY (nothing reads them; gradients unchanged)
 *   "afau_head_split" (default 0 = by launch size): the cross-set attention's 16 heads per 16-row
 *                block split over 1 / 2 / 4 / 8 / 16 workgroups (same results)
 *   "scatter_batch" (FPM_SCATTER_BATCH, default 4): out-edges whose loads the scatter SplineConv
 *                backward issues together (1 or 4; same sums, same order)
 * Switches whose variants round differently (results within fp32 rounding, not bit-identical):
 *   "sinkhorn_fast" (FPM_SINKHORN_FAST, default 1): shifted single-pass lse after the first step
 *       (0 = max-shifted lse every step; 2 = 1 with scalar loads in the n > 256 streaming kernel)
 *   "sinkhorn_lform" (default 1): Sinkhorn forward for n <= 256 on the L-form register kernel
 *       (the log matrix as the tile, lse subtracted per step) or on the potential-form kernel (0)
 *   "topk_fast" (FPM_TOPK_FAST, default 1): shifted single-pass early soft top-k column steps */
int fpm_set_tuning(const char* key, int value);

/* ---- SplineConv message passing ---------------------------------------------------------------
 * Replaces PyG 1.6.3 SplineConv(768, 768, dim=2, kernel_size=5, aggr='max') inside SConv /
 * SiameseSConvOnNodes (src/model/spline_conv.py:17, 28-57).
 * fpm_spline_plan: per-node cell masks, (node, cell) product rows ranked per cell, GEMM tile table
 * and the dst CSR (device workspace of fpm_spline_plan_bytes bytes; reused by both layers and by
 * the GNN layer's CSR).
 * fpm_spline_conv_fwd: one layer; mode & 1 == 0 -> relu(conv(x)), mode & 1 == 1 -> xres + 0.1 * conv(x).
 * mode >> 1 (bf16 out_t, inference): out_t rows split for a near-fp32 bf16-MFMA product, 2304 columns
 * per row, hi = bf16(z), lo = bf16(z - hi): 1 -> [hi | lo | hi] (A operand), 2 -> [hi | hi | lo] (B).
 * W: (26, 768 out, 768 in) = the 25 spline-cell weights transposed, then the root weight
 * transposed; y_ws: fpm_spline_y_bytes(dtype, E, num_nodes) bytes of product-row scratch. */
long fpm_spline_plan_bytes(long E, long num_nodes);
long fpm_spline_y_bytes(int dtype, long E, long num_nodes);
int fpm_spline_plan(const int* src, const int* dst, const float* pseudo, long E, long num_nodes, int nmax, void* ws,
                    long ws_bytes, void* stream);
/* the same plan built one workgroup per graph (LDS sort / counts instead of device-wide atomics)
 * when every graph has <= max_graph_edges <= 4096 edges and 26 <= nmax <= 1024; otherwise (or
 * max_graph_edges <= 0) it is fpm_spline_plan.  Graphs' edges must be contiguous ranges in graph
 * order (every batch builder emits them so).  Bit-identical plan. */
int fpm_spline_plan_graphs(const int* src, const int* dst, const float* pseudo, long E, long num_nodes, int nmax,
                           long max_graph_edges, void* ws, long ws_bytes, void* stream);
int fpm_spline_plan_csr(void* ws, long E, long num_nodes, int** dst_ptr, int** nbr_local);
/* several per-graph plans (e.g. every pipeline chunk of one side of a batch) by one launch of each
 * plan kernel.  jobs: device array of njobs records of fpm_spline_plan_job_bytes() (= 56) bytes,
 * {const int* src; const int* dst; const float* pseudo; long E, num_nodes, ws_off;
 *  int ngraphs, gstart}: job j's inputs, its first graph's index among all jobs' graphs
 * (gstart, ascending; total_graphs = the sum of ngraphs) and the 256-aligned offset of its plan
 * (fpm_spline_plan_bytes(E, num_nodes) bytes) in ws.  Every job must meet fpm_spline_plan_graphs'
 * per-graph conditions (graphs of <= 4096 edges as contiguous ranges, num_nodes = ngraphs nmax,
 * 26 <= nmax <= 1024).  Each plan equals fpm_spline_plan_graphs of that job alone. */
int fpm_spline_plan_multi(const void* jobs, int njobs, int total_graphs, int nmax, void* ws, void* stream);
int fpm_spline_plan_job_bytes(void);
int fpm_spline_conv_fwd(int dtype, const void* x_op, const void* plan_ws, long E, long num_nodes, int nmax,
                        const int* nvalid, const void* W, const float* bias, void* y_ws, long y_ws_bytes, int mode,
                        const float* xres, const float* cscale, float* out_f, void* out_t, void* stream);
/* the same, also writing argmax[num_nodes][768] (int32: CSR slot of the in-edge attaining each
 * channel's max, the first in CSR order; -1 without in-edges) for fpm_spline_conv_bwd_data_scatter
 * (the training forward) */
int fpm_spline_conv_fwd_argmax(int dtype, const void* x_op, const void* plan_ws, long E, long num_nodes, int nmax,
                               const int* nvalid, const void* W, const float* bias, void* y_ws, long y_ws_bytes,
                               int mode, const float* xres, const float* cscale, float* out_f, void* out_t,
                               int* argmax, void* stream);
/* probe x gallery (C4): broadcast the shared source graph's SplineConv output y (rows x 768 fp32)
 * to B pairs: out_f[b] = y, out_t[b] = dtype(y o coef[b]) (coef may be NULL) -- the same values the
 * per-pair path's fused epilogue writes; split (bf16 only) as fpm_spline_conv_fwd's mode >> 1. */
int fpm_rows_bcast_scale(int dtype, const float* y, long rows, int B, const float* coef, float* out_f, void* out_t,
                         int split, void* stream);
/* vertex_attr_to_edge_attr (spline_conv.py:73-81): out[e] = x[src[e]] - x[dst[e]] */
int fpm_edge_diff(const float* x, const int* src, const int* dst, long E, int D, float* out, void* stream);
/* same, written into a padded per-pair layout and scaled: out[row[e]] = (x[src]-x[dst]) o c[pair[e]]
 * (Xe * coefficients of the quadratic affinity, ngm.py:282-289 / affinity_layer.py:15); cscale may
 * be NULL.  Feeds the optional Ke GEMM (fpm_gemm epilogue EPI_HALF_AFFINITY = 4). */
int fpm_edge_diff_padded(const float* x, const int* src, const int* dst, const int* pair, const int* row,
                         const float* cscale, long E, int D, float* out, void* stream);

/* ---- association-graph GNN layer --------------------------------------------------------------
 * Replaces PYGNNLayer.forward's SAGEConv mean aggregation over the Kronecker pattern + MLPs +
 * classifier (src/model/gnn.py:207-218; pattern from factorize_graph_matching.py:57-95 and
 * gmdataset.py:614-642), factorised so the n1*n2 x n1*n2 pattern is never built.
 * X: (B, C, n2max, n1max) with C in {1, 17}; Xout channels 0..15 and zbuf (B, n2max, n1max)
 * are written; the caller runs fpm_sinkhorn_log_fwd(zbuf -> Xout channel 16).  Last layer: pass
 * vpart (B, n2max, n1max) and the final classifier weights cls_w (17): vpart = cls_w[0:16] . x1
 * is written instead of Xout channels 0..15 (fpm_node_classifier then reads vpart + channel 16).
 * params: fpm_gnn_param_count(C) floats = lin_l.weight^T [C][16], lin_l.bias [16],
 * lin_r.weight^T [C][16], n_self_func.0.weight^T [C][16], n_self_func.0.bias [16],
 * n_self_func.2.weight^T [16][16], n_self_func.2.bias [16], classifier.weight [16], classifier.bias.
 * n1max <= 1024; neighbour lists ascending (the plan CSR). */
int fpm_kron_gnn_layer_fwd(const float* X, int C, int B, int n1max, int n2max, const int* ptr1, const int* nbr1,
                           const int* ptr2, const int* nbr2, const int* n1, const int* n2, const float* params,
                           float* Xout, float* zbuf, float* vpart, const float* cls_w, void* stream);
/* The same with a block order: the k-th workgroup of pair b takes graph-2 node ord2[b * n2max + k]
 * (a permutation of 0..n2max-1 per pair; NULL = identity).  Same results (a schedule only). */
int fpm_kron_gnn_layer_fwd_ord(const float* X, int C, int B, int n1max, int n2max, const int* ptr1,
                               const int* nbr1, const int* ptr2, const int* nbr2, const int* n1, const int* n2,
                               const float* params, float* Xout, float* zbuf, float* vpart, const float* cls_w,
                               const int* ord2, void* stream);
int fpm_gnn_param_count(int C);
/* final classifier (ngm.py:368-369): s[b][i][j] = w . X[b][:, j, i] + bias; with vpart (NULL =
 * all 17 channels): s = vpart + w[16] X[b][16, j, i] + bias */
int fpm_node_classifier(const float* X, int B, int n1max, int n2max, const float* w, const float* bias,
                        const float* vpart, float* s, void* stream);

/* ---- AFA-U k regressor (ngm.py:386-412, src/model/afau.py) ------------------------------------
 * crossset_attn: the row block's multi-head cross-set attention (afau.py:99-142) -> out rows of
 * 256 = 16 heads x 16; dtype 0 = fp32, 1 = bf16, 2 = split bf16 rows [hi | lo | hi] (768 wide, the
 * A operand of the near-fp32 combine product, see fpm_split_bf16x3).  stats (optional, training):
 * per (pair, row, head) the softmax's (max score, sum of exp(score - max)), float2[B][n1max][16]. */
int fpm_crossset_attn_fwd(int dtype, const float* cost, long c_sb, long c_ld, int B, int n1max, int n2max,
                          const int* n2, const float* Wv, int emb, const float* mix1w, const float* mix1b,
                          const float* mix2w, const float* mix2b, void* out, float* stats, void* stream);
int fpm_instnorm(int dtype, const float* in1, const float* in2, int B, int P, int Cn, const int* nvalid,
                 const float* onehot_bias, const float* w, const float* bias, float eps, float* out_f, void* out_t,
                 int ldt, float* gmax, void* stream);
int fpm_afau_head(const float* gr, const float* gc, int B, int E, const float* r0w, const float* r0b,
                  const float* r2w, const float* r2b, const float* c0w, const float* c0b, const float* c2w,
                  const float* c2b, float* ks, void* stream);

/* ---- fp64 k chain (csrc/precise.hip) ----------------------------------------------------------
 * Everything after the vertex affinity Kp in double precision, for small boxes where k_prob is
 * ill-conditioned (Net.k_f64_nmax): the same algebra as the fp32 entry points above.
 * fpm_kron_gnn_layer_fwd_f64: PYGNNLayer (gnn.py:207-226); X is fp32 Kp (x_f64 = 0, C = 1) or the
 *   fp64 state (x_f64 = 1, C = 17); params as fpm_kron_gnn_layer_fwd; Xout channels 0..15 and zbuf
 *   fp64; n1max <= 1024 and C x n1max doubles within LDS.
 * fpm_sinkhorn_log_fwd_f64: pygm sinkhorn (sinkhorn.py:85-87) in fp64 on fp32 (s_f64 = 0) or fp64
 *   input, any strides; o64 (fp64) and / or o32 (fp32 copy) outputs; boxes up to 128 x 128.
 * fpm_node_classifier_f64: s = classifier(emb) (ngm.py:368-369) -> s64 (+ optional fp32 s32).
 * fpm_crossset_attn_row_f64: the AFA-U row block's attention with R0 = 0 (afau.py:231-300), out
 *   (B x n1max) x 256 fp64.
 * fpm_gemm_f64: C = act(A W^T + bias), relu = 1 for ReLU (the AFA-U projections and FFN).
 * fpm_instnorm_f64: AddAndInstanceNormalization (afau.py:154-176) over P positions; in1 (+ in2) or
 *   (in1 NULL) the col block's one-hot + onehot_bias; out and / or gmax (max over positions).
 * fpm_afau_head_f64: ks[b] = sigmoid((final_row(gr[b]) + final_col(gc[cidx[b]])) / 2) (ngm.py:401-412),
 *   cidx NULL = b; ks fp32.
 * fpm_soft_topk_fwd_f64: soft_topk (soft_topk.py:8-53, 166-255) incl. the while loop in fp64 from the
 *   fp64 ss -> ds_mat fp32 (and an optional second, e.g. pinned host, copy); ws >= 2 B n1max n2max
 *   doubles; steps_out (optional) = steps taken. */
int fpm_kron_gnn_layer_fwd_f64(const void* X, int x_f64, int C, int B, int n1max, int n2max, const int* ptr1,
                               const int* nbr1, const int* ptr2, const int* nbr2, const int* n1, const int* n2,
                               const float* params, double* Xout, double* zbuf, void* stream);
int fpm_sinkhorn_log_fwd_f64(const void* s, int s_f64, long s_sb, long s_si, long s_sj, double* o64, long o_sb,
                             long o_si, long o_sj, float* o32, long f_sb, long f_si, long f_sj, const int* n1,
                             const int* n2, int B, int n1max, int n2max, int iters, double tau, int dummy_row,
                             void* stream);
int fpm_node_classifier_f64(const double* X, int B, int n1max, int n2max, const float* w, const float* bias,
                            double* s64, float* s32, void* stream);
int fpm_crossset_attn_row_f64(const double* cost, long c_sb, long c_ld, int B, int n1max, int n2max, const int* n2,
                              const double* Wv, int emb, const double* mix1w, const double* mix1b,
                              const double* mix2w, const double* mix2b, double* out, void* stream);
int fpm_gemm_f64(const double* A, int lda, const double* W, int ldw, const double* bias, double* C, int ldc, int M,
                 int N, int K, int relu, void* stream);
int fpm_instnorm_f64(const double* in1, const double* in2, int B, int P, int Cn, const int* nvalid,
                     const double* onehot_bias, const double* w, const double* bias, double eps, double* out,
                     double* gmax, void* stream);
int fpm_afau_head_f64(const double* gr, const double* gc, const int* cidx, int B, int E, const double* r0w,
                      const double* r0b, const double* r2w, const double* r2b, const double* c0w, const double* c0b,
                      const double* c2w, const double* c2b, float* ks, void* stream);
int fpm_soft_topk_fwd_f64(const double* ss, long s_sb, long s_ld, const int* n1, const int* n2, const float* k, int B,
                          int n1max, int n2max, int iters, double tau, double* ws, long ws_doubles, float* out,
                          long o_sb, long o_ld, int* steps_out, float* out2, long o2_sb, long o2_ld, void* stream);

/* ---- AFA-U backward (training, src/model/afau.py:54-300 through ks_loss, training_loop.py:60) ---
 * fpm_afau_head_bwd: ks = sigmoid((final_row(gr) + final_col(gc)) / 2) -> dgr, dgc (B x E) and
 *   per-pair parameter partials part[b] = 2 x [dW0 (8 x E) | db0 (8) | dw2 (8) | db2] (row, col).
 * fpm_instnorm_bwd: InstanceNorm1d over positions (afau.py:154-176), input in1 (+ in2) or the col
 *   block's one-hot + bias; seed dy (dense) or gseed (max-pool gradient routed to the argmax);
 *   dx (optional, accumulate) and per-pair dw / db partials (B x Cn).
 * fpm_afau_attn_bwd: the row block's cross-set attention (afau.py:231-300 with R0 = 0) given the
 *   forward's output and softmax stats: per-pair dWv partials (B x 256 x n2max) and mixed-score
 *   partials (B x 16 x 49 = [dW2 | dW1 row 1 | db1 | db2]).
 * fpm_rows_sum: out[u][k] (+)= sum_b in[b][k] in order over the b with key[b] == u, or (key NULL)
 *   over the u-th of nkeys contiguous row chunks (deterministic).
 * fpm_transpose: out[c][r] = in[r][c], rows [R, ldo) of out zero.
 * fpm_elementwise: mode 0 x *= (ref > 0) (ReLU backward), mode 1 x += ref. */
int fpm_afau_head_bwd(const float* gr, const float* gc, int B, int E, const float* r0w, const float* r0b,
                      const float* r2w, const float* r2b, const float* c0w, const float* c0b, const float* c2w,
                      const float* c2b, const float* dks, float* dgr, float* dgc, float* part, void* stream);
int fpm_instnorm_bwd(const float* in1, const float* in2, int B, int P, int Cn, const int* nvalid,
                     const float* onehot_bias, const float* w, const float* bias, float eps, const float* dy,
                     const float* gseed, float* dx, int accumulate, float* dw_part, float* db_part, void* stream);
int fpm_afau_attn_bwd(const float* cost, long c_sb, long c_ld, int B, int n1max, int n2max, const int* n2,
                      const float* Wv, int emb, const float* mix1w, const float* mix1b, const float* mix2w,
                      const float* mix2b, const float* att_out, const float* datt, const float* stats,
                      float* dwv_part, float* mix_part, void* stream);
int fpm_rows_sum(const float* in, int B, long K, const int* key, int nkeys, float* out, int accumulate,
                 void* stream);
int fpm_transpose(const float* in, long R, int C, long ldi, float* out, long ldo, void* stream);
int fpm_elementwise(float* x, const float* ref, long n, int mode, void* stream);

/* ---- GNN weight-gradient reductions (training, gnn.py:207-226 parameters) --------------------
 * part[w][o * (C + ones) + c] over fpm_outer_sum_parts(B, N) rows w: per-workgroup partial sums of
 * U[b][o][p] V[b][c][p] (and of U[b][o][p] alone in column C when ones != 0); strides in elements;
 * O <= 32, C <= 17.  The caller sums the rows (fpm_rows_sum). */
long fpm_outer_sum_parts(int B, long N);
int fpm_outer_sum(const float* U, long sUb, long sUo, int O, const float* V, long sVb, long sVc, int Cc, int ones,
                  int B, long N, float* part, void* stream);

/* ---- MatchClassifier training: BatchNorm2d(train) fused with the ReLU before it ---------------
 * (ngm.py:90-99 conv -> ReLU -> BatchNorm2d blocks; torch F.batch_norm(training=True) semantics)
 * x: conv output (N, C, HW) fp32; y = BN(relu(x)) with batch statistics; stats (2C floats):
 * (mean, invstd) for the backward; running_mean / running_var (nullable): momentum update with the
 * unbiased variance.  Backward: dx = d/dx through the BN and the ReLU, dgamma, dbeta (C).
 * ws: fpm_bn_ws_floats(N, C) floats.  Reductions are deterministic. */
long fpm_bn_ws_floats(int N, int C);
int fpm_bn_relu_train_fwd(const float* x, int N, int C, long HW, const float* gamma, const float* beta, float eps,
                          float momentum, float* running_mean, float* running_var, float* y, float* stats, float* ws,
                          void* stream);
int fpm_bn_relu_train_bwd(const float* x, const float* dy, int N, int C, long HW, const float* gamma,
                          const float* stats, float* dx, float* dgamma, float* dbeta, float* ws, void* stream);

/* ---- MatchClassifier (ngm.py:75-106, applied at :451-455) -------------------------------------
 * dtype 0: conv2 on fp32 matrix cores (exact fp32 products, parity mode); 1: conv2 operands in
 * bf16 (fp32 accumulation, the bf16 throughput mode). */
long fpm_match_cls_ws_floats(int B, int H, int W);
int fpm_match_cls_fwd(int dtype, const float* s, const float* perm, int B, int H, int W, const float* w1,
                      const float* b1, const float* bn1_sc, const float* bn1_sh, const float* w2, const float* b2,
                      const float* bn2_sc, const float* bn2_sh, const float* fcw, const float* fcb, float* ws,
                      float* logits, float* prob, void* stream);

/* ---- MatchClassifier in training (ngm.py:75-106 under model.train(), train.py's classifier stages)
 * Both BatchNorm2d layers in train mode (batch statistics, biased variance; running buffers get the
 * momentum update with the unbiased variance), MaxPool2d's first-maximum gradient routing, ReLU's
 * [x > 0] gate.  s, perm: (B, H, W) fp32 contiguous (the classifier input is s * perm; perm carries
 * no gradient).  Forward: logits (B); saved: fpm_match_cls_train_ws_floats(B, H, W, 0) floats kept
 * for the backward; ws: (.., 1) floats.  Backward: for dlogits (B) -> ds (B, H, W) and every
 * parameter gradient (overwritten); ws: (.., 2) floats.  Replaces the MIOpen convolutions and the
 * torch max-pool / BatchNorm kernels of the training step; reductions are deterministic. */
long fpm_match_cls_train_ws_floats(int B, int H, int W, int which);
int fpm_match_cls_train_fwd(const float* s, const float* perm, int B, int H, int W, const float* w1,
                            const float* b1, const float* g1, const float* be1, float* rm1, float* rv1,
                            const float* w2, const float* b2, const float* g2, const float* be2, float* rm2,
                            float* rv2, const float* fcw, const float* fcb, float eps, float momentum, float* saved,
                            float* ws, float* logits, void* stream);
int fpm_match_cls_train_bwd(const float* s, const float* perm, int B, int H, int W, const float* w1, const float* b1,
                            const float* g1, const float* w2, const float* b2, const float* g2, const float* fcw,
                            const float* saved, const float* dlogits, float* ws, float* ds, float* dw1, float* db1,
                            float* dg1, float* dbe1, float* dw2, float* db2, float* dg2, float* dbe2, float* dfcw,
                            float* dfcb, void* stream);

/* ---- API parity: the reference's sparse extension ops (off the live forward path) ------------
 * Replace src/extension/sparse_dot/sparse_dot.cpp:322-331 (csr_dot_csc_to_dense,
 * dense_dot_csc_to_dense, csr_dot_diag_to_csr; csr_dot_csc_to_csr is CPU-only in the reference)
 * and src/extension/bilinear_diag/bilinear_diag.cpp:324-326 (bilinear_diag).  Batched CSR/CSC in
 * the csx_matrix.py:20-93 layout: int64 indices, int64 indptr of length B*len+1 with global
 * offsets.  dtype: 0 f32, 2 f64, 3 f16 (device); 0 f32, 2 f64 (host).  Caller allocates outputs;
 * the dense outputs are fully written (no pre-zeroing needed). */
int fpm_csr_dot_csc_to_dense(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                             const long* t2_indices, const long* t2_indptr, const void* t2_data, long batch_size,
                             long out_h, long out_w, void* out, void* stream);
int fpm_dense_dot_csc_to_dense(int dtype, const void* t1, const long* t2_indices, const long* t2_indptr,
                               const void* t2_data, long batch_size, long out_h, long out_w, long t1_w, void* out,
                               void* stream);
int fpm_csr_dot_diag_to_csr(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                            const void* t2, long batch_size, long out_h, long out_w, void* out_data, void* stream);
int fpm_bilinear_diag(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data, const void* t2,
                      long feat_size, const long* t3_indices, const long* t3_indptr, const void* t3_data,
                      long batch_size, long xlen, void* out, void* stream);
/* host twins (CPU tensors, synchronous); csr_dot_csc_to_csr: call with out_indices == NULL for the
 * nnz (out_indptr filled if given), then with buffers of capacity >= nnz.  Returns nnz or -1. */
long fpm_csr_dot_csc_to_csr_host(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                                 const long* t2_indices, const long* t2_indptr, const void* t2_data, long batch_size,
                                 long out_h, long out_w, long* out_indptr, long capacity, long* out_indices,
                                 void* out_data);
int fpm_csr_dot_diag_to_csr_host(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                                 const void* t2, long batch_size, long out_h, long out_w, void* out_data);
int fpm_bilinear_diag_host(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                           const void* t2, long feat_size, const long* t3_indices, const long* t3_indptr,
                           const void* t3_data, long batch_size, long xlen, void* out);

/* ---- Gconv (src/model/gcn.py:8-38; unused by Net) ----------------------------
 * out = norm1(A) relu(x Wa^T + ba) + relu(x Wu^T + bu); W = [Wa; Wu] (2*dout, din), bias likewise;
 * ws: fpm_gconv_ws_floats(B, n, dout) floats. */
long fpm_gconv_ws_floats(int B, int n, int dout);
int fpm_gconv_fwd(const float* A, const float* x, int B, int n, int din, int dout, const float* W, const float* bias,
                  int norm, float* ws, float* out, void* stream);

/* ---- on-device graph construction ------------------------------------------
 * Replaces the DataLoader-side utils/build_graphs.py:12-120 (build_graphs / delaunay_triangulate /
 * fully_connect, sym=True), GMDataset.to_pyg_graph (src/gmdataset.py:170-189) and the collate's
 * Kronecker index lists (src/gmdataset.py:614-642).  G graphs of padded size nmax <= 1024.
 * fpm_graph_build: P (G, nmax, 2) fp32 keypoints, n (G) int32; strategy 0 = 'tri' (Delaunay),
 *   1 = 'fc', 2 = 'near' (edges longer than thre removed).  Writes adj (G, nmax, W) uint32 bit rows
 *   (W = fpm_graph_words(nmax)), deg (G, nmax) int32 out-degrees, ecount (G) int32 and, if Adense
 *   is not NULL, the dense adjacency (G, nmax, nmax) fp32 of build_graphs.
 * fpm_graph_edges: edge list in np.nonzero(A) order with node ids g*nmax + i: src/dst (sum E)
 *   int32, pseudo (sum E, 2) = clip(0.5*(P_src-P_dst)/rescale + 0.5, 0, 1); edge_off (G+1) int64
 *   (may be NULL); Ginc/Hinc (G, nmax, epad) fp32 incidence matrices, caller-zeroed (may be NULL).
 * fpm_kron_pattern: one pair's (rowG, colH) = (CSCMatrix3d(kron(G2,G1)).indices,
 *   CSCMatrix3d(kron(H2,H1)).transpose().indices) over E1*E2 edge pairs; node ids minus base1/base2;
 *   out_dtype 0 = float32, 1 = int64. */
int fpm_graph_words(int nmax);
int fpm_graph_build(const float* P, const int* n, int G, int nmax, int strategy, double thre, uint32_t* adj, int* deg,
                    int* ecount, float* Adense, void* stream);
int fpm_graph_edges(const float* P, const uint32_t* adj, const int* deg, const int* ecount, int G, int nmax,
                    double rescale, int* src, int* dst, float* pseudo, long* edge_off, float* Ginc, float* Hinc,
                    int epad, void* stream);
int fpm_kron_pattern(const int* src1, const int* dst1, long E1, const int* src2, const int* dst2, long E2, int base1,
                     int base2, int n1pad, int out_dtype, void* rowG, void* colH, void* stream);

/* ---- image front end after the CNN (ngm.py:235-248) -----------------------
 * Replaces normalize_over_channels (ngm.py:65-67) + utils/feature_align.py:5-126 (bilinear gather at
 * the keypoints, with its (H, W) vs (320, 240) scale mix and border nearest-neighbour branch) +
 * concat_features (ngm.py:70-72) + the AdaptiveMaxPool2d(1) global feature (feature_extractor.py:62).
 * nodes/edges: (B, C, H, W) fp32 maps given by shape[4] and element strides[4] (NCHW or
 * channels_last); P (B, nmax, 2) fp32 keypoints in the ori_w x ori_h frame; n (B) int32.
 * X (B*nmax, ldx) fp32 rows = [U (C_nodes) || F (C_edges)], zero rows past n[b];
 * wglob (B, C_edges) fp32 (may be NULL); ws: fpm_feature_align_ws_floats(...) floats. */
long fpm_feature_align_ws_floats(const long* node_shape, const long* edge_shape);
int fpm_feature_align_fwd(const float* nodes, const long* node_shape, const long* node_stride, const float* edges,
                          const long* edge_shape, const long* edge_stride, const float* P, const int* n, int nmax,
                          float ori_w, float ori_h, float* ws, float* X, long ldx, float* wglob, void* stream);
/* Its backward (train.py stages 1 / 3 / 5 train the backbone through this stage, ngm.py:235-251):
 * dX (B*nmax, ldx) and dwglob (B, C_edges, may be NULL) -> dnodes / dedges (the maps' shapes, own
 * element strides), every element written: transpose of the bilinear gather (keypoints found per
 * pixel in a fixed order, no atomics), the channel-norm backward, and the global max-pool gradient
 * at each (image, channel)'s first maximum.  ws: the forward's workspace (pixel norms); nmax <= 4096,
 * C_nodes, C_edges <= 512. */
int fpm_feature_align_bwd(const float* nodes, const long* node_shape, const long* node_stride, const float* edges,
                          const long* edge_shape, const long* edge_stride, const float* P, const int* n, int nmax,
                          float ori_w, float ori_h, const float* ws, const float* dX, long ldx, const float* dwglob,
                          float* dnodes, const long* dnode_stride, float* dedges, const long* dedge_stride,
                          void* stream);

/* ---- profiling hooks: HIP-event timing of the dominant kernel (edge-message GEMM) ------------ */
int fpm_profile_enable(int on);
int fpm_profile_enabled(void);   /* 1 while enabled: Net.run then launches eagerly (no HIP graphs) */
int fpm_profile_read(double* ms_total, double* flops_total, int* count);

/* ---- device: batched linear sum assignment -------------------------------
 * The host solver's algorithm (utils/hungarian.py:8-66 -> scipy LSAP, csrc/lsa.cpp) restated for
 * one wavefront per pair with identical arithmetic, scan order and tie rule: assignments are
 * bit-identical to fpm_lsa_batch_host.  s: device float32, batch stride sb, row stride ld; maximise
 * s over each n1[b] x n2[b] block.  assign (B, n1max) int32 (column or -1); status (B) int32:
 * 0 ok, 1 infeasible, 2 NaN / -inf cost.  n1max, n2max <= 1024.  Asynchronous on stream. */
int fpm_lsa_batch_device(const float* s, long sb, long ld, const int* n1, const int* n2, int B, int n1max, int n2max,
                         int* assign, int* status, void* stream);

/* ---- training backward ----------------------------------------------------
 * Vector-Jacobian products of the forward ops above for train.py's stages
 * (src/train/training_loop.py:32-60: PermutationLoss(ds_mat) + ks_loss + cls_loss, .backward()).
 * The reference gets these from autograd through PyG / torch_sparse / pygmtools / torch ops.
 *
 * Sinkhorn (sinkhorn.py:85-87 -> pygm.sinkhorn): s and dp are strided (B, n1max, n2max) views of
 * the forward's input and of the gradient of its output; ds (contiguous box) receives d/ds, zero
 * outside each valid block.  ws: fpm_sinkhorn_bwd_ws_floats(...) floats.  Deterministic. */
long fpm_sinkhorn_bwd_ws_floats(int B, int n1max, int n2max, int iters);
int fpm_sinkhorn_log_bwd(const float* s, long s_sb, long s_si, long s_sj, const float* dp, long d_sb, long d_si,
                         long d_sj, float* ds, const int* n1, const int* n2, int B, int n1max, int n2max, int iters,
                         float tau, int dummy_row, float* ws, long ws_floats, void* stream);
/* soft top-k (soft_topk.py:23-45 + Sinkhorn_m.forward_log :166-255, incl. the continuation):
 * ss / k / steps as given to / returned by fpm_soft_topk_fwd; dds: gradient of ds_mat; dss
 * (contiguous box) receives d/dss (anchor min/max share split over ties like torch's min()/max()).
 * status[b] = 1 if the forward ran more steps than the replay holds (4096).  No gradient for k. */
long fpm_soft_topk_bwd_ws_floats(int B, int n1max, int n2max);
int fpm_soft_topk_bwd(const float* ss, long sb, long ld, const int* n1, const int* n2, const float* k,
                      const int* steps, int B, int n1max, int n2max, float tau, const float* dds, long db, long dld,
                      float* dss, float* ws, long ws_floats, int* status, void* stream);
/* SplineConv layer w.r.t. its input (PyG SplineConv aggr='max' under SConv, spline_conv.py:17,
 * 33-38): mode 0 = conv 0 + F.relu (hout = the layer's output), mode 1 = conv 1 under the Siamese
 * residual (x + 0.1 * conv).  y_ws: the forward's product rows of this layer; Wb: (26, 768 in,
 * 768 out) = the reference's weight layout then root, operand dtype.  dY (fp32, fpm_spline_y_bytes
 * of dtype 0) receives the product-row gradients (the weight gradient is X_rows^T dY per cell, row
 * ranges from fpm_spline_plan_rows); dY_op: bf16 copy (dtype 1); dXrows: fp32 like dY; dX (num_nodes,
 * 768) fp32, overwritten or accumulated. */
int fpm_spline_plan_rows(void* plan_ws, long E, long num_nodes, int** arows, int** cell_off);
int fpm_spline_conv_bwd_data(int dtype, const void* plan_ws, long E, long num_nodes, int nmax, const int* nvalid,
                             const void* Wb, const void* y_ws, int mode, const float* gout, const float* hout,
                             float* dY, void* dY_op, float* dXrows, float* dX, int accumulate, void* stream);
/* the same without atomics: rplan_ws = the plan of the reversed edges (its CSR lists every node's
 * out-edges), argmax from fpm_spline_conv_fwd_argmax; one workgroup per source node accumulates its
 * product rows' gradients in LDS over its out-edges in a fixed order (deterministic, no memset).
 * dtype 1: the cell rows' gradients land in dY_op only and dY holds the root rows (the bias
 * gradient) -- fpm_set_tuning("scatter_f32_rows", 1) writes the fp32 cell rows too. */
int fpm_spline_conv_bwd_data_scatter(int dtype, const void* plan_ws, const void* rplan_ws, const int* argmax, long E,
                                     long num_nodes, int nmax, const int* nvalid, const void* Wb, const void* y_ws,
                                     int mode, const float* gout, const float* hout, float* dY, void* dY_op,
                                     float* dXrows, float* dX, int accumulate, void* stream);
/* out[c][q] = rows[q] >= 0 ? in[rows[q]][c] : 0 (c < C, q < Q; dtype 0 fp32, 1 bf16): K-major
 * copies of the gathered node rows / product-row gradients for the per-cell SplineConv weight
 * gradients dW_cell = X_rows^T dY_rows, run as fpm_gemm batches of fixed K chunks. */
int fpm_gather_transpose(int dtype, const void* in, long ldi, const int* rows, long Q, int C, void* out, long ldo,
                         void* stream);
/* SplineConv weight operands for a training step (spline_conv.py:28-57 weights change every step):
 * the K cells weight[k] (Cin x Cout, the reference layout) and root (Cin x Cout) stacked as K + 1
 * matrices into out, transposed to [k][Cout][Cin] (transpose = 1, the forward GEMM's B) or kept
 * [k][Cin][Cout] (0, the backward's B); dtype 0 fp32, 1 bf16.  One pass per copy. */
int fpm_spline_weight_pack(const float* weight, const float* root, int K, int Cin, int Cout, int transpose, int dtype,
                           void* out, void* stream);
/* Factorised Kronecker SAGE-mean aggregation alone (SAGEConv mean over the association pattern,
 * gnn.py:208 / ngm.py:339-344): adjoint = 0 recomputes the forward's agg (T = in-edge CSRs);
 * adjoint = 1 with T = out-edge CSRs is its transpose (dX = A1^T (dagg / den) A2 + D o dagg / den).
 * q1, q2: in-edge CSR pointers (degrees for den).  X / out: (B, C, n2max, n1max) fp32.
 * adjoint | 2: add the result into out instead of storing it (the backward's dX += adjoint). */
int fpm_kron_agg(const float* X, int C, int B, int n1max, int n2max, const int* tptr1, const int* tnbr1,
                 const int* tptr2, const int* tnbr2, const int* q1, const int* q2, const int* n1, const int* n2,
                 int adjoint, float* out, void* stream);

/* PYGNNLayer node MLPs + classifier, per association node (gnn.py:208-215 transposed): given dXn
 * (gradient of [x1 || S], (B, 17, n2max, n1max)) and dz (gradient of the classifier logit, i.e.
 * the Sinkhorn backward of channel 16), writes dX = W1^T dh1 + Wr^T dx1 and dagg = Wl^T dx1
 * ((B, C, ...)), and V = [dx1 | dh1 | dm | h1] ((B, 64, N)) for the weight-gradient reductions.
 * params: the forward's packed layer parameters. */
int fpm_kron_gnn_layer_bwd_point(const float* X, int C, int B, int n1max, int n2max, const float* dXn, const float* dz,
                                 const float* params, float* dX, float* dagg, float* V, void* stream);

/* ---- host: batched linear sum assignment ------------------------------------------------------
 * Replaces utils/hungarian.py:8-66 (scipy linear_sum_assignment on -s, per pair).  Synchronous,
 * HOST memory, nthreads worker threads.  assign[b][r] = column or -1.  Returns 0 or (pair + 1).
 * Solver path chosen once per process from the CPU: AVX-512 F/DQ/VL/BW -> float cost rows read
 * in place with the tie rule resolved in the scan pass (default); FPM_LSA_DENSE512=1 / FPM_LSA_AVX2=1
 * / FPM_LSA_SCALAR=1 force the older dense-scan or scalar solvers.  All paths return scipy's
 * assignment bit for bit (tests/test_lsa_isa.py). */
int fpm_lsa_batch_host(const float* s, long sb, long ld, const int* n1, const int* n2, int B, int n1max, int* assign,
                       int nthreads);
/* Asynchronous form (the pipelined forward's Hungarian): fpm_lsa_submit queues the batch on
 * nthreads persistent workers that serve pairs first-in first-out across batches and returns a
 * ticket > 0 (the pointers must stay valid until the wait); fpm_lsa_wait(ticket, block, seconds)
 * returns 0 / failing pair + 1 like fpm_lsa_batch_host and releases the ticket, -2 while the batch
 * is still running when block == 0, -1 for an unknown ticket; seconds (optional) receives the
 * batch's span on the workers. */
long fpm_lsa_submit(const float* s, long sb, long ld, const int* n1, const int* n2, int B, int n1max, int* assign,
                    int nthreads);
int fpm_lsa_wait(long ticket, int block, double* seconds);

#ifdef __cplusplus
}
#endif
#endif /* FPM_H_ */
