// C-ABI entry for the generic (batched, optionally row-gathered) MFMA GEMM with fused epilogues.
// Used by: SplineConv root term, global-weight coefficient (affinity_layer.py:13), vertex
// affinity Kp (affinity_layer.py:15-18), AFA-U projections/FFN (afau.py:99-103,188-199).
#include "gemm_phase.h"
#include "gemm_pp.h"
#include <cstdlib>
#include <cstring>

namespace fpm {
int& gemm_bn256_min();
}

extern "C" int fpm_gemm(int dtype, const void* A, long lda, long sA, const int* a_rows, const void* B, long ldb,
                        long sB, int M, int N, int K, int batch, int epi, const float* bias, float* Cf, void* Ct,
                        long ldc, long sC, const int* n1, const int* n2, void* stream) {
    using namespace fpm;
    FPM_CHECK_ARG(dtype == 0 || dtype == 1, "gemm: dtype must be 0 (f32) or 1 (bf16)");
    FPM_CHECK_ARG(M >= 0 && N > 0 && K > 0 && batch >= 0, "gemm: bad sizes M=%d N=%d K=%d", M, N, K);
    FPM_CHECK_ARG(K % (dtype ? 8 : 4) == 0, "gemm: K=%d must be a multiple of %d", K, dtype ? 8 : 4);
    FPM_CHECK_ARG(lda % (dtype ? 8 : 4) == 0 && ldb % (dtype ? 8 : 4) == 0, "gemm: lda/ldb must keep rows 16-B aligned");
    FPM_CHECK_ARG((epi != EPI_AFFINITY && epi != EPI_HALF_AFFINITY) || (n1 && n2),
                  "gemm: affinity epilogues need n1/n2");
    FPM_CHECK_ARG(epi >= EPI_STORE && epi <= EPI_HALF_AFFINITY, "gemm: bad epilogue %d", epi);
    if (M == 0 || batch == 0) return 0;
    GemmParams p = {};
    p.A = A; p.lda = lda; p.sA = sA; p.a_rows = a_rows;
    p.B = B; p.ldb = ldb; p.sB = sB; p.sB_seg = 0;
    p.row_scale = nullptr;
    p.M = M; p.N = N; p.K = K; p.nseg = 1;
    p.tile_info = nullptr; p.group_off = nullptr;
    p.epi = epi; p.bias = bias; p.Cf = Cf; p.Ct = Ct; p.ldc = ldc; p.sC = sC; p.n1 = n1; p.n2 = n2;
    hipStream_t st = (hipStream_t)stream;
    // bf16 with a large M: the 256-row LDS-DMA tiles (gemm_big.h)
    const int mt = (M + G2_BM - 1) / G2_BM;
    const bool epi_ok = epi == EPI_STORE || epi == EPI_RELU || (epi == EPI_AFFINITY && Cf && !Ct);
    const bool big = dtype == 1 && M >= G2_BM && K % G2_BK == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
                     !(Cf && Ct) && (Cf ? ldc % 4 == 0 : ldc % 8 == 0) && epi_ok &&
                     (long)mt * ((N + 127) / 128) * batch >= 128;
    if (big) {
        // 256-wide tiles once they alone give >= gemm_bn256_min workgroups (FPM_GEMM_BN256_MIN)
        const int BN = (N % 256 == 0 && (long)mt * (N / 256) * batch >= gemm_bn256_min()) ? 256 : 128;
        p.remap_mtiles = mt;
        dim3 grid(remap_grid_big(N, BN, mt), 1, batch);
        const bool f32 = Cf != nullptr;
        const bool phase = BN == 256 && use_gemm_phase(K);
#define FPM_BIG(BN_, E_, F_)                                                                            \
    do {                                                                                               \
        if (BN_ == 256 && phase) hipLaunchKernelGGL((gemm_phase_kernel<E_, F_>), grid, dim3(G2_THREADS), 0, st, p); \
        else hipLaunchKernelGGL((gemm_big_kernel<BN_, E_, F_>), grid, dim3(G2_THREADS), 0, st, p);      \
    } while (0)
        if (epi == EPI_AFFINITY) {
            if (BN == 256) FPM_BIG(256, EPI_AFFINITY, true); else FPM_BIG(128, EPI_AFFINITY, true);
        } else if (BN == 256) {
            if (epi == EPI_RELU) { if (f32) FPM_BIG(256, EPI_RELU, true); else FPM_BIG(256, EPI_RELU, false); }
            else { if (f32) FPM_BIG(256, EPI_STORE, true); else FPM_BIG(256, EPI_STORE, false); }
        } else {
            if (epi == EPI_RELU) { if (f32) FPM_BIG(128, EPI_RELU, true); else FPM_BIG(128, EPI_RELU, false); }
            else { if (f32) FPM_BIG(128, EPI_STORE, true); else FPM_BIG(128, EPI_STORE, false); }
        }
#undef FPM_BIG
        return check_launch("fpm_gemm");
    }
    p.remap_mtiles = (M + GBM - 1) / GBM;
    dim3 grid(remap_grid(N, p.remap_mtiles), 1, batch);
    if (dtype == 0) hipLaunchKernelGGL((gemm_kernel<float, false>), grid, dim3(GTHREADS), 0, st, p);
    else hipLaunchKernelGGL((gemm_kernel<bf16_t, false>), grid, dim3(GTHREADS), 0, st, p);
    return check_launch("fpm_gemm");
}

namespace fpm {
// FPM_GEMM_PP: the product GEMM on the two-workgroups-per-CU 256 x 128 kernel (gemm_pp.h)
int& gemm_pp_flag() {
    static int on = [] {
        const char* e = getenv("FPM_GEMM_PP");
        return e ? atoi(e) : 0;
    }();
    return on;
}

int& gemm_phase_flag() {
    static int on = [] {
        const char* e = getenv("FPM_GEMM_PHASE");
        return e ? atoi(e) : 1;
    }();
    return on;
}

int& gemm_bn256_min() {
    static int v = [] {
        const char* e = getenv("FPM_GEMM_BN256_MIN");
        return e ? atoi(e) : 512;
    }();
    return v;
}
}  // namespace fpm

// AFA-U encoder block tail (afau.py:188-199 + the max over positions): gmax[b][n] =
// max_p InstanceNorm_p(res[b*P + p][n] + (A W^T)[b*P + p][n] + bias[n]) * nw[n] + nb[n], P = 256
// positions per pair = one 256-row tile (EPI_NORM_MAX epilogue of gemm_big_kernel<128>).
extern "C" int fpm_gemm_norm_max(const void* A, long lda, const void* B, long ldb, int M, int N, int K,
                                 const float* bias, const float* res, long ldres, const float* nw, const float* nb,
                                 float eps, int P, float* gmax, void* stream) {
    using namespace fpm;
    FPM_CHECK_ARG(P == G2_BM || 2 * P == G2_BM, "gemm_norm_max: P=%d must be %d or %d (one or two pairs per tile)", P,
                  G2_BM, G2_BM / 2);
    FPM_CHECK_ARG(M >= 0 && M % P == 0 && N > 0 && K > 0 && K % G2_BK == 0, "gemm_norm_max: bad sizes M=%d N=%d K=%d",
                  M, N, K);
    FPM_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0 && ldres >= N, "gemm_norm_max: bad strides");
    FPM_CHECK_ARG(res && nw && nb && gmax, "gemm_norm_max: null operand");
    if (M == 0) return 0;
    GemmParams p = {};
    p.A = A; p.lda = lda; p.B = B; p.ldb = ldb;
    p.M = M; p.N = N; p.K = K; p.nseg = 1;
    p.epi = EPI_NORM_MAX; p.bias = bias; p.ldc = ldres;
    p.res = res; p.nw = nw; p.nb = nb; p.eps = eps; p.gmax = gmax; p.norm_p = P;
    const int mt = (M + G2_BM - 1) / G2_BM;
    p.remap_mtiles = mt;
    dim3 grid(remap_grid_big(N, 128, mt), 1, 1);
    hipLaunchKernelGGL((gemm_big_kernel<128, EPI_NORM_MAX, true>), grid, dim3(G2_THREADS), 0, (hipStream_t)stream, p);
    return fpm::check_launch("fpm_gemm_norm_max");
}

// AFA-U encoder block head (afau.py:188-199 first InstanceNorm1d on the attention-combine output):
// out_f = InstanceNorm_p((A W^T)[b*P + p] + bias) * nw + nb over each pair's P = 256 rows (one GEMM
// tile, EPI_NORM_OUT epilogue), out_t (optional) its bf16 copy with row stride ldt and zero columns
// [N, ldt) -- the combine output never reaches HBM un-normalised.
extern "C" int fpm_gemm_norm_out(const void* A, long lda, const void* B, long ldb, int M, int N, int K,
                                 const float* bias, const float* nw, const float* nb, float eps, int P, float* out_f,
                                 long ldc, void* out_t, long ldt, void* stream) {
    using namespace fpm;
    FPM_CHECK_ARG(P == G2_BM || 2 * P == G2_BM, "gemm_norm_out: P=%d must be %d or %d (one or two pairs per tile)", P,
                  G2_BM, G2_BM / 2);
    FPM_CHECK_ARG(M >= 0 && M % P == 0 && N > 0 && N % 4 == 0 && K > 0 && K % G2_BK == 0,
                  "gemm_norm_out: bad sizes M=%d N=%d K=%d", M, N, K);
    FPM_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0 && ldc >= N && ldc % 4 == 0 && (!out_t || (ldt >= N && ldt % 4 == 0 &&
                  ldt <= ((N + 127) / 128) * 128)), "gemm_norm_out: bad strides");
    FPM_CHECK_ARG(nw && nb && out_f, "gemm_norm_out: null operand");
    if (M == 0) return 0;
    GemmParams p = {};
    p.A = A; p.lda = lda; p.B = B; p.ldb = ldb;
    p.M = M; p.N = N; p.K = K; p.nseg = 1;
    p.epi = EPI_NORM_OUT; p.bias = bias; p.Cf = out_f; p.ldc = ldc; p.Ct = out_t; p.ldt = ldt;
    p.nw = nw; p.nb = nb; p.eps = eps; p.norm_p = P;
    const int mt = (M + G2_BM - 1) / G2_BM;
    p.remap_mtiles = mt;
    dim3 grid(remap_grid_big(N, 128, mt), 1, 1);
    hipLaunchKernelGGL((gemm_big_kernel<128, EPI_NORM_OUT, true>), grid, dim3(G2_THREADS), 0, (hipStream_t)stream, p);
    return fpm::check_launch("fpm_gemm_norm_out");
}

// Near-fp32 operands for the next product (the AFA-U encoder in the gate-passing bf16x3 mode,
// afau.py:99-103,188-199): C = epi(A W^T + bias) in fp32 on the 256-row bf16 MFMA tile, stored as
// split bf16 rows out_t3 = [hi | lo | hi] (segment stride Kp, columns [N, Kp) of each segment zero,
// row stride ldt >= 3 Kp: exactly fpm_split_bf16x3 of the fp32 result) and, if out_f is given, as
// fp32 rows too.  epi: EPI_STORE / EPI_RELU, or EPI_NORM_OUT (InstanceNorm over each pair's P = 256
// rows, weights nw / nb; out_f required) -- the fp32 intermediate never makes its own HBM pass.
extern "C" int fpm_gemm_x3out(const void* A, long lda, const void* B, long ldb, int M, int N, int K, int epi,
                              const float* bias, const float* nw, const float* nb, float eps, int P, float* out_f,
                              long ldc, void* out_t3, long ldt, int Kp, void* stream) {
    using namespace fpm;
    FPM_CHECK_ARG(epi == EPI_STORE || epi == EPI_RELU || epi == EPI_NORM_OUT, "gemm_x3out: bad epilogue %d", epi);
    FPM_CHECK_ARG(M >= 0 && N > 0 && N % 4 == 0 && K > 0 && K % G2_BK == 0, "gemm_x3out: bad sizes M=%d N=%d K=%d",
                  M, N, K);
    FPM_CHECK_ARG(Kp >= N && Kp % 4 == 0 && Kp <= ((N + 127) / 128) * 128 && ldt >= 3L * Kp && ldt % 4 == 0,
                  "gemm_x3out: segment Kp=%d must be in [N, N rounded up to 128], 4-aligned, ldt >= 3 Kp", Kp);
    FPM_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0 && (!out_f || (ldc >= N && ldc % 4 == 0)), "gemm_x3out: bad strides");
    FPM_CHECK_ARG(out_t3, "gemm_x3out: null out_t3");
    FPM_CHECK_ARG(epi != EPI_NORM_OUT || ((P == G2_BM || 2 * P == G2_BM) && M % P == 0 && nw && nb && out_f),
                  "gemm_x3out: the norm epilogue needs P = %d or %d rows per pair, nw, nb and out_f", G2_BM, G2_BM / 2);
    if (M == 0) return 0;
    GemmParams p = {};
    p.A = A; p.lda = lda; p.B = B; p.ldb = ldb;
    p.M = M; p.N = N; p.K = K; p.nseg = 1;
    p.epi = epi; p.bias = bias; p.Cf = out_f; p.ldc = ldc; p.Ct = out_t3; p.ldt = ldt; p.split = Kp;
    p.nw = nw; p.nb = nb; p.eps = eps; p.norm_p = epi == EPI_NORM_OUT ? P : 0;
    const int mt = (M + G2_BM - 1) / G2_BM;
    p.remap_mtiles = mt;
    dim3 grid(remap_grid_big(N, 128, mt), 1, 1);
    hipStream_t st = (hipStream_t)stream;
    if (epi == EPI_NORM_OUT) hipLaunchKernelGGL((gemm_big_kernel<128, EPI_NORM_OUT, true>), grid, dim3(G2_THREADS), 0, st, p);
    else if (epi == EPI_RELU) hipLaunchKernelGGL((gemm_big_kernel<128, EPI_RELU, true>), grid, dim3(G2_THREADS), 0, st, p);
    else hipLaunchKernelGGL((gemm_big_kernel<128, EPI_STORE, true>), grid, dim3(G2_THREADS), 0, st, p);
    return check_launch("fpm_gemm_x3out");
}

namespace {
// Xc[b * nmax + i][k] = X[b * nmax + i][k] * coef[b][k]  (X o c of affinity_layer.py:15)
__global__ __launch_bounds__(256) void rows_scale_kernel(const float* __restrict__ X, long ldx, int nmax, int d,
                                                         const float* __restrict__ coef, float* __restrict__ Xc) {
    const long r = blockIdx.x;
    const int b = (int)(r / nmax);
    for (int k = threadIdx.x; k < d; k += 256) Xc[r * d + k] = X[r * ldx + k] * coef[(long)b * d + k];
}
}  // namespace

// The vertex / edge affinity of InnerProductWithWeightsAffinity._forward (affinity_layer.py:11-19)
// under the surveyed name: per pair b, c = tanh(A_w w[b] + A_b) (a GEMM with the
// tanh epilogue), then K[b][i][j] = epi(((X1[b] o c) X2[b]^T)[i][j]) on the valid n1[b] x n2[b]
// block and 0 outside it, epi 0 = softplus(v) - 0.5 (vertex, ngm.py:277-280), 1 = 0.5 (softplus(v) -
// 0.5) (edge, ngm.py:282-287).  fp32 throughout (the forward's own bf16 path fuses these steps into
// the SplineConv epilogue and the GNN-layout Kp GEMM).  X1: (B n1max, d) rows (stride ld1), X2:
// (B n2max, d) (ld2), w: (B, kw) global weights, A_w: (d, kw), K: (B, n1max, n2max) (row stride ldk,
// batch stride n1max * ldk).  ws: caller workspace of fpm_affinity_ws_floats(B, n1max, d) floats.
extern "C" long fpm_affinity_ws_floats(int B, int n1max, int d) { return (long)B * d + (long)B * n1max * d; }

extern "C" int fpm_affinity_fwd(const float* X1, long ld1, const float* X2, long ld2, const float* w, int kw,
                                const float* A_w, const float* A_b, int B, int n1max, int n2max, int d, const int* n1,
                                const int* n2, int epi, float* K, long ldk, float* ws, long ws_floats, void* stream) {
    using namespace fpm;
    FPM_CHECK_ARG(epi == 0 || epi == 1, "affinity_fwd: epi must be 0 (vertex) or 1 (edge)");
    FPM_CHECK_ARG(B >= 0 && n1max > 0 && n2max > 0 && d > 0 && d % 4 == 0 && kw > 0 && kw % 4 == 0,
                  "affinity_fwd: bad sizes");
    FPM_CHECK_ARG(ld1 >= d && ld2 >= d && ld2 % 4 == 0 && ldk >= n2max, "affinity_fwd: bad strides");
    FPM_CHECK_ARG(ws && ws_floats >= fpm_affinity_ws_floats(B, n1max, d), "affinity_fwd: workspace too small");
    FPM_CHECK_ARG(n1 && n2 && K && X1 && X2 && w && A_w, "affinity_fwd: null operand");
    if (B == 0) return 0;
    float* coef = ws;
    float* X1c = ws + (long)B * d;
    if (fpm_gemm(0, w, kw, 0, nullptr, A_w, kw, 0, B, d, kw, 1, EPI_TANH, A_b, coef, nullptr, d, 0, nullptr, nullptr,
                 stream))
        return 1;
    hipLaunchKernelGGL(rows_scale_kernel, dim3((unsigned)((long)B * n1max)), dim3(256), 0, (hipStream_t)stream, X1,
                       ld1, n1max, d, coef, X1c);
    if (check_launch("fpm_affinity_fwd")) return 1;
    // rows i (graph 1) x columns j (graph 2); the affinity epilogue masks rows by its n2 argument and
    // columns by its n1 argument, so the pair sizes are passed crosswise
    return fpm_gemm(0, X1c, d, (long)n1max * d, nullptr, X2, ld2, (long)n2max * ld2, n1max, n2max, d, B,
                    epi == 0 ? EPI_AFFINITY : EPI_HALF_AFFINITY, nullptr, K, nullptr, ldk, (long)n1max * ldk, n2, n1,
                    stream);
}

int& plan_graph_flag();
int& combine_npb_flag();
int& sinkhorn_bwd_reg_flag();
int& sinkhorn_fast_flag();
int& sinkhorn_lform_flag();
int& soft_topk_fast_flag();
int& afau_attn_v_flag();
int& gnn_store_sc1_flag();
int& combine_store_sc1_flag();
int& gemm_store_sc1_flag();
int& combine_lds_kb_flag();
int& gnn_mlp_off_flag();
int& outer_sum_vec_flag();
int& gnn_sweeps_flag();
int& scatter_f32_rows_flag();
int& scatter_batch_flag();
int& afau_head_split_flag();

extern "C" int fpm_set_tuning(const char* key, int value) {
    int* f = nullptr;
    if (key && !strcmp(key, "gemm_phase")) f = &fpm::gemm_phase_flag();
    else if (key && !strcmp(key, "gemm_pp")) f = &fpm::gemm_pp_flag();
    else if (key && !strcmp(key, "plan_graph")) f = &plan_graph_flag();
    else if (key && !strcmp(key, "combine_npb")) f = &combine_npb_flag();
    else if (key && !strcmp(key, "sinkhorn_bwd_reg")) f = &sinkhorn_bwd_reg_flag();
    else if (key && !strcmp(key, "sinkhorn_fast")) f = &sinkhorn_fast_flag();
    else if (key && !strcmp(key, "sinkhorn_lform")) f = &sinkhorn_lform_flag();
    else if (key && !strcmp(key, "topk_fast")) f = &soft_topk_fast_flag();
    else if (key && !strcmp(key, "afau_attn_v")) f = &afau_attn_v_flag();
    else if (key && !strcmp(key, "gnn_store_sc1")) f = &gnn_store_sc1_flag();
    else if (key && !strcmp(key, "combine_store_sc1")) f = &combine_store_sc1_flag();
    else if (key && !strcmp(key, "gemm_store_sc1")) f = &gemm_store_sc1_flag();
    else if (key && !strcmp(key, "combine_lds_kb")) f = &combine_lds_kb_flag();
    else if (key && !strcmp(key, "gnn_mlp_off")) f = &gnn_mlp_off_flag();
    else if (key && !strcmp(key, "outer_sum_vec")) f = &outer_sum_vec_flag();
    else if (key && !strcmp(key, "gnn_sweeps")) f = &gnn_sweeps_flag();
    else if (key && !strcmp(key, "scatter_f32_rows")) f = &scatter_f32_rows_flag();
    else if (key && !strcmp(key, "scatter_batch")) f = &scatter_batch_flag();
    else if (key && !strcmp(key, "afau_head_split")) f = &afau_head_split_flag();
    if (!f) {
        fpm::set_error("fpm_set_tuning: unknown key '%s'", key ? key : "(null)");
        return -1;
    }
    // timing probes that make results wrong are refused unless the process opted in explicitly
    if (f == &gnn_mlp_off_flag() && value != 0) {
        const char* e = getenv("FPM_TIMING_PROBES");
        if (!e || strcmp(e, "1") != 0) {
            fpm::set_error("fpm_set_tuning: '%s' is a timing probe with wrong results; set FPM_TIMING_PROBES=1 "
                           "to allow it", key);
            return -1;
        }
    }
    const int prev = *f;
    *f = value;
    return prev;
}

// f32 -> bf16 conversion (operand copies for the bf16 MFMA path)
namespace {
__global__ void cast_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    long stride = (long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) y[i] = fpm::f2bf(x[i]);
}

// 8 values per thread: two 16-B loads, one 16-B store (the scalar form ran at ~1.6 TB/s with 2-B
// stores); same rounding, bit-identical
__global__ __launch_bounds__(256) void cast_bf16_v8_kernel(const float4* __restrict__ x, uint4* __restrict__ y, long n8) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n8) return;
    const float4 a = x[2 * i], b = x[2 * i + 1];
    uint4 o;
    o.x = (uint32_t)fpm::f2bf(a.x) | ((uint32_t)fpm::f2bf(a.y) << 16);
    o.y = (uint32_t)fpm::f2bf(a.z) | ((uint32_t)fpm::f2bf(a.w) << 16);
    o.z = (uint32_t)fpm::f2bf(b.x) | ((uint32_t)fpm::f2bf(b.y) << 16);
    o.w = (uint32_t)fpm::f2bf(b.z) | ((uint32_t)fpm::f2bf(b.w) << 16);
    y[i] = o;
}
}  // namespace

extern "C" int fpm_cast_bf16(const float* x, void* y, long n, void* stream) {
    if (n <= 0) return 0;
    if (n % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
        const long n8 = n / 8;
        hipLaunchKernelGGL(cast_bf16_v8_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           (const float4*)x, (uint4*)y, n8);
        return fpm::check_launch("fpm_cast_bf16");
    }
    long blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(cast_bf16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, (bf16_t*)y, n);
    return fpm::check_launch("fpm_cast_bf16");
}

// Global weights of each pair, normalize_over_channels(cat(w1[b], w2[b])) (ngm.py:65-67, 262-268):
// one 256-thread workgroup per pair; the sum of squares is reduced in a fixed order (per-thread
// strided partials, then a fixed LDS tree), so a pair's result does not depend on how many pairs
// share the launch -- a shard or a pipeline chunk computed alone reproduces its slice exactly.
namespace {
__global__ __launch_bounds__(256) void global_weights_kernel(const float* __restrict__ w1, long ld1,
                                                             const float* __restrict__ w2, long ld2, int D1, int D2,
                                                             float* __restrict__ out, long ldo) {
    __shared__ float red[256];
    const int b = blockIdx.x, t = threadIdx.x;
    const float* a = w1 + (long)b * ld1;
    const float* c = w2 + (long)b * ld2;
    float acc = 0.f;
    for (int i = t; i < D1 + D2; i += 256) {
        const float v = i < D1 ? a[i] : c[i - D1];
        acc = fmaf(v, v, acc);
    }
    red[t] = acc;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h) red[t] += red[t + h];
        __syncthreads();
    }
    const float nrm = sqrtf(red[0]);
    float* o = out + (long)b * ldo;
    for (int i = t; i < D1 + D2; i += 256) o[i] = (i < D1 ? a[i] : c[i - D1]) / nrm;
}
}  // namespace

extern "C" int fpm_global_weights(const float* w1, long ld1, const float* w2, long ld2, int B, int D1, int D2,
                                  float* out, long ldo, void* stream) {
    FPM_CHECK_ARG(B >= 0 && D1 >= 0 && D2 >= 0 && ld1 >= D1 && ld2 >= D2 && ldo >= D1 + D2,
                  "global_weights: bad sizes");
    if (B == 0) return 0;
    hipLaunchKernelGGL(global_weights_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, w1, ld1, w2, ld2, D1, D2,
                       out, ldo);
    return fpm::check_launch("fpm_global_weights");
}

// Affinity coefficients c[b][n] = tanh(sum_k g[b][k] WT[k][n] + bias[n]) (affinity_layer.py:13, the
// global-weight projection) for the B pairs of a forward: B x 768 outputs over K = 1024 -- too few
// 128 x 128 GEMM tiles to fill the chip at small B (6 workgroups at B = 128, ~0.12 ms).  A workgroup
// = 64 columns n (lanes; WT rows read coalesced, [K][N] layout) x 4 K-quarters (waves) x R pairs
// with their g rows in LDS: each wave runs one fp32 fma chain over its quarter (k ascending, 16
// weight loads in flight), the four partial sums are added in quarter order -- a fixed reduction
// per output, so a pair's coefficients are the same whatever batch they are computed in.
namespace {
constexpr int COEF_KMAX = 1024, COEF_Q = 4;
template <int COEF_R>
__global__ __launch_bounds__(256) void coef_tanh_kernel(const float* __restrict__ g, long ldg,
                                                        const float* __restrict__ wT, const float* __restrict__ bias,
                                                        int B, int K, int N, float* __restrict__ out, long ldo) {
    __shared__ float gs[COEF_R][COEF_KMAX];
    __shared__ float part[COEF_Q][COEF_R][64];
    const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int n = blockIdx.x * 64 + lane, b0 = blockIdx.y * COEF_R;
    for (int i = threadIdx.x; i < COEF_R * K; i += 256) {
        const int r = i / K, k = i - r * K;
        gs[r][k] = b0 + r < B ? g[(long)(b0 + r) * ldg + k] : 0.f;
    }
    __syncthreads();
    const int nc = n < N ? n : N - 1;                     // clamped column: loads stay in bounds
    const int kq = (K + COEF_Q - 1) / COEF_Q, kb = q * kq, ke = kb + kq < K ? kb + kq : K;
    float acc[COEF_R];
#pragma unroll
    for (int r = 0; r < COEF_R; ++r) acc[r] = 0.f;
    const float* w = wT + nc;
    for (int k0 = kb; k0 < ke; k0 += 16) {
        float wv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) wv[u] = k0 + u < ke ? w[(long)(k0 + u) * N] : 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (k0 + u < ke)
#pragma unroll
                for (int r = 0; r < COEF_R; ++r) acc[r] = fmaf(gs[r][k0 + u], wv[u], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < COEF_R; ++r) part[q][r][lane] = acc[r];
    __syncthreads();
    if (q != 0 || n >= N) return;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < COEF_R; ++r) {
        float v = part[0][r][lane];
#pragma unroll
        for (int j = 1; j < COEF_Q; ++j) v += part[j][r][lane];
        if (b0 + r < B) out[(long)(b0 + r) * ldo + n] = tanhf(v + bv);
    }
}
}  // namespace

extern "C" int fpm_coef_tanh(const float* g, long ldg, const float* wT, const float* bias, int B, int K, int N,
                             float* out, long ldo, void* stream) {
    FPM_CHECK_ARG(B >= 0 && K > 0 && K <= COEF_KMAX && N > 0 && ldg >= K && ldo >= N, "coef_tanh: bad sizes");
    if (B == 0) return 0;
    // R pairs per workgroup: 2 at small B (enough workgroups to fill the chip), 8 from 256 pairs on
    // (each workgroup re-reads its 64 weight columns; at R = 2 and B = 1024 that was ~1.6 GB of L2
    // reads, 0.107 ms); the per-output reduction does not depend on R
    if (B >= 256)
        hipLaunchKernelGGL(coef_tanh_kernel<8>, dim3((unsigned)((N + 63) / 64), (unsigned)((B + 7) / 8)), dim3(256), 0,
                           (hipStream_t)stream, g, ldg, wT, bias, B, K, N, out, ldo);
    else
        hipLaunchKernelGGL(coef_tanh_kernel<2>, dim3((unsigned)((N + 63) / 64), (unsigned)((B + 1) / 2)), dim3(256), 0,
                           (hipStream_t)stream, g, ldg, wT, bias, B, K, N, out, ldo);
    return fpm::check_launch("fpm_coef_tanh");
}

// Split-bf16 operand rows for near-fp32 GEMMs on the bf16 MFMA path: x = hi + lo with hi = bf16(x)
// and lo = bf16(x - hi); dst row = [hi | lo | hi] (each segment Kp wide, zero in [K, Kp)), to be
// multiplied by weights packed as [B_hi | B_hi | B_lo] along K, which sums hi*B_hi + lo*B_hi +
// hi*B_lo (the dropped lo*B_lo term is ~2^-16 of the product) with fp32 accumulation.
namespace {
__global__ __launch_bounds__(256) void split_bf16x3_kernel(const float* __restrict__ src, long lds, int K, int Kp,
                                                           bf16_t* __restrict__ dst, long ldd) {
    const long r = blockIdx.x;
    const float* a = src + r * lds;
    bf16_t* o = dst + r * ldd;
    for (int k = threadIdx.x; k < Kp; k += 256) {
        const float v = k < K ? a[k] : 0.f;
        const bf16_t hi = fpm::f2bf(v);
        const bf16_t lo = fpm::f2bf(v - fpm::bf2f(hi));
        o[k] = hi;
        o[Kp + k] = lo;
        o[2 * Kp + k] = hi;
    }
}
}  // namespace

extern "C" int fpm_split_bf16x3(const float* src, long lds, long rows, int K, int Kp, void* dst, long ldd,
                                void* stream) {
    FPM_CHECK_ARG(rows >= 0 && K > 0 && Kp >= K && lds >= K && ldd >= 3L * Kp, "split_bf16x3: bad sizes");
    if (rows == 0) return 0;
    hipLaunchKernelGGL(split_bf16x3_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, src, lds, K, Kp,
                       (bf16_t*)dst, ldd);
    return fpm::check_launch("fpm_split_bf16x3");
}

