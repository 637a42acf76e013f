// fp64 k chain: the forward from the vertex affinity Kp to k_prob in double precision
// (reference ngm.py:326-412: PYGNNLayer x3 gnn.py:207-226, the readout ngm.py:368-369, the final
// Sinkhorn ngm.py:371 / sinkhorn.py:85-87, and the AFA-U regressor afau.py:54-300).
//
// Why: on image-derived matcher inputs k_prob is ill-conditioned.  The AFA-U instance norms divide
// by the across-row spread of nearly uniform attention outputs, and the tau = 0.01 Sinkhorns
// multiply every upstream rounding by 100, so k moves by ~1e-4 under the fp32 rounding of ANY
// stage after Kp (tools/kprob_arith.py, profiles/r06_kprob_arith_cpu.txt: the fp32 reference sits
// up to 2e-4 from its own fp64 value at n = 32, 3.6e-5 at n = 192).  The product path therefore
// evaluates this chain in fp64 when the padded box is small (Net.k_f64_nmax, default 64 keypoints),
// where it costs little.  The products before it (SplineConv, Kp) stay fp32: their rounding moves
// k by < 5e-6.
//
// Kernels (all plain fp64 VALU; the boxes are at most 128 keypoints, so every kernel is
// latency-bound and small):
//   gnn_layer_f64_kernel   the factorised Kronecker SAGE mean + node MLPs + classifier (the same
//                          algebra as gnn.hip), state X[b][c][d][i] in fp64
//   sinkhorn_f64_kernel    pygm's log-domain Sinkhorn, one workgroup per pair, the block in LDS
//   classifier_f64_kernel  s = classifier(emb) (ngm.py:368-369), fp64 and fp32 copies
//   attn_row_f64_kernel    the row block's cross-set attention with R0 = 0 (afau.py:231-300)
//   gemm_f64_kernel        C = act(A W^T + bias): the AFA-U projections / FFN
//   instnorm_f64_kernel    AddAndInstanceNormalization (+ max over positions)
//   afau_head_f64_kernel   final_row / final_col + sigmoid(mean) (ngm.py:401-412)
//   soft_topk_f64_kernel   soft top-k's 2-column Sinkhorn incl. the while loop -> ds_mat (fp32 out)
#include "fpm_common.h"

namespace {

// same block order as gnn.hip: the blocks of pair b run on XCD b % 8
__device__ __forceinline__ bool pair_block64(int n2max, int B, int& b, int& d) {
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    b = (k / n2max) * 8 + x;
    d = k % n2max;
    return b < B;
}

// packed layer parameters (fp32, gnn.hip's GnnPack): WlT[C][16] bl[16] WrT[C][16] W1T[C][16] b1[16]
// W2T[16][16] b2[16] wc[16] bc
template <int C>
struct Pack64 {
    static constexpr int Wl = 0, bl = Wl + 16 * C, Wr = bl + 16, W1 = Wr + 16 * C, b1 = W1 + 16 * C, W2 = b1 + 16,
                         b2 = W2 + 256, wc = b2 + 16, bc = wc + 16, total = bc + 1;
};

// One workgroup per (pair b, graph-2 node d), one thread per graph-1 node i.
//   agg[c] = ( sum_{a in N1(i)} sum_{e in N2(d)} X[c][e][a] + D X[c][d][i] ) / (deg1(i) deg2(d) + D),
//   D = [d*n1max + i < n1b*n2b]  (the padded-space diagonal, quirk A.10(ii))
//   x1 = lin_l(agg) + lin_r(x) + relu(W2 relu(W1 x + b1) + b2),   z = classifier(x1)
// Phase 1 stages T[c][i] = sum_{e in N2(d)} X[c][e][i] in LDS; phase 2 gathers over N1(i).
template <int C, typename TIn>
__global__ __launch_bounds__(1024) void gnn_layer_f64_kernel(const TIn* __restrict__ X, int n1max, int n2max,
                                                             const int* __restrict__ ptr1, const int* __restrict__ nbr1,
                                                             const int* __restrict__ ptr2, const int* __restrict__ nbr2,
                                                             const int* __restrict__ n1, const int* __restrict__ n2,
                                                             const float* __restrict__ W, double* __restrict__ Xo,
                                                             double* __restrict__ zbuf, int B) {
    using P = Pack64<C>;
    extern __shared__ double T64[];
    int b, d;
    if (!pair_block64(n2max, B, b, d)) return;
    const int i = threadIdx.x;
    const long N = (long)n1max * n2max;
    const TIn* Xb = X + (long)b * C * N;
    const int b2 = ptr2[(long)b * n2max + d], e2 = ptr2[(long)b * n2max + d + 1];
    if (i < n1max) {
        for (int c = 0; c < C; ++c) {
            double t = 0.0;
            for (int e = b2; e < e2; ++e) t += (double)Xb[(long)c * N + (long)nbr2[e] * n1max + i];
            T64[c * n1max + i] = t;
        }
    }
    __syncthreads();
    if (i >= n1max) return;
    const long p = (long)d * n1max + i;
    const int beg = ptr1[(long)b * n1max + i], end = ptr1[(long)b * n1max + i + 1];
    const bool self = p < (long)n1[b] * n2[b];
    const double cnt = (double)((end - beg) * (e2 - b2) + (self ? 1 : 0));
    double x[C], agg[C];
    for (int c = 0; c < C; ++c) {
        x[c] = (double)Xb[(long)c * N + p];
        double a = 0.0;
        for (int e = beg; e < end; ++e) a += T64[c * n1max + nbr1[e]];
        if (self) a += x[c];
        agg[c] = cnt > 0.0 ? a / cnt : 0.0;
    }
    double h[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        double s = (double)W[P::b1 + m];
        for (int c = 0; c < C; ++c) s = fma((double)W[P::W1 + c * 16 + m], x[c], s);
        h[m] = s > 0.0 ? s : 0.0;
    }
    double z = (double)W[P::bc];
    double* Xob = Xo + (long)b * 17 * N;
#pragma unroll
    for (int o = 0; o < 16; ++o) {
        double l = (double)W[P::bl + o], r = 0.0, t = (double)W[P::b2 + o];
        for (int c = 0; c < C; ++c) {
            l = fma((double)W[P::Wl + c * 16 + o], agg[c], l);
            r = fma((double)W[P::Wr + c * 16 + o], x[c], r);
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) t = fma((double)W[P::W2 + m * 16 + o], h[m], t);
        const double x1 = l + r + (t > 0.0 ? t : 0.0);
        Xob[(long)o * N + p] = x1;
        z = fma((double)W[P::wc + o], x1, z);
    }
    zbuf[(long)b * N + p] = z;
}

// pygmtools sinkhorn (log domain, batched_operation=False), restated in fp64: L = s[:r, :c] / tau,
// run transposed when r > c, dummy rows of -100 up to a square when asked, then alternately
// L -= logsumexp over the row / over the column, NaN -> -inf; out = exp(L[:r]) on the valid block,
// 0 elsewhere.  One workgroup per pair; the (rows x cols) block in LDS (ld = cols + 1), one thread per
// line for the reductions.
template <typename TIn>
__global__ __launch_bounds__(256) void sinkhorn_f64_kernel(const TIn* __restrict__ s, long s_sb, long s_si, long s_sj,
                                                           double* __restrict__ o64, long o_sb, long o_si, long o_sj,
                                                           float* __restrict__ o32, long f_sb, long f_si, long f_sj,
                                                           const int* __restrict__ n1, const int* __restrict__ n2,
                                                           int n1max, int n2max, int iters, double tau, int dummy) {
    extern __shared__ double L[];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int r = n1[b], c = n2[b];
    const bool tr = r > c;
    const int R0 = tr ? c : r, Cc = tr ? r : c;
    const int Rt = (dummy && Cc > R0) ? Cc : R0;
    const int ld = Cc + 1;
    const double NEG = -__builtin_inf();
    for (int q = tid; q < Rt * Cc; q += blockDim.x) {
        const int i = q / Cc, j = q % Cc;
        double v;
        if (i < R0) {
            const long off = (long)b * s_sb + (tr ? (long)j * s_si + (long)i * s_sj : (long)i * s_si + (long)j * s_sj);
            v = (double)s[off] / tau;
        } else {
            v = -100.0;
        }
        L[i * ld + j] = v;
    }
    __syncthreads();
    for (int it = 0; it < iters; ++it) {
        const bool rows = (it & 1) == 0;
        const int nl = rows ? Rt : Cc, len = rows ? Cc : Rt;
        const int step = rows ? 1 : ld, lstride = rows ? ld : 1;
        for (int ln = tid; ln < nl; ln += blockDim.x) {
            double* v = L + (long)ln * lstride;
            double m = NEG;
            for (int k = 0; k < len; ++k) m = fmax(m, v[k * step]);
            double lse = NEG;
            if (m != NEG) {
                double sum = 0.0;
                for (int k = 0; k < len; ++k) sum += exp(v[k * step] - m);
                lse = m + log(sum);
            }
            for (int k = 0; k < len; ++k) {
                const double y = v[k * step] - lse;
                v[k * step] = y != y ? NEG : y;
            }
        }
        __syncthreads();
    }
    for (int q = tid; q < n1max * n2max; q += blockDim.x) {
        const int i = q / n2max, j = q % n2max;
        double v = 0.0;
        if (i < r && j < c) v = exp(tr ? L[j * ld + i] : L[i * ld + j]);
        if (o64) o64[(long)b * o_sb + (long)i * o_si + (long)j * o_sj] = v;
        if (o32) o32[(long)b * f_sb + (long)i * f_si + (long)j * f_sj] = (float)v;
    }
}

// s[b][i][j] = bias + sum_c w[c] X[b][c][j][i]  (ngm.py:368-369; v.view(B, n2max, n1max).transpose)
__global__ __launch_bounds__(256) void classifier_f64_kernel(const double* __restrict__ X, int n1max, int n2max,
                                                             const float* __restrict__ w, const float* __restrict__ bias,
                                                             double* __restrict__ s64, float* __restrict__ s32, int B) {
    const long N = (long)n1max * n2max;
    const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (long)B * N) return;
    const int b = (int)(q / N);
    const long p = q % N;                 // p = j * n1max + i
    const int j = (int)(p / n1max), i = (int)(p % n1max);
    const double* Xb = X + (long)b * 17 * N;
    double v = (double)bias[0];
    for (int c = 0; c < 17; ++c) v = fma((double)w[c], Xb[(long)c * N + p], v);
    const long o = (long)b * N + (long)i * n2max + j;
    s64[o] = v;
    if (s32) s32[o] = (float)v;
}

// Row-block cross-set attention with R0 = 0 (afau.py:231-300): q = 0, so the mixed score of head h is
//   m_h(c) = mix2_bias[h] + sum_k mix2[h][k] relu(mix1[h][1][k] c + mix1_bias[h][k])
// of the cost c = ss[b][i][j] over all n2max columns; out[h*16+d] = sum_{j < n2b} softmax_j(m) Wv[h*16+d][j]
// (v = Wv C0: column j of Wv for j < n2b, 0 for the padded columns).  One workgroup per (pair, row),
// thread t = (head t / 16, lane t % 16); the scores in LDS.
__global__ __launch_bounds__(256) void attn_row_f64_kernel(const double* __restrict__ cost, long c_sb, long c_ld,
                                                           int n1max, int n2max, const int* __restrict__ n2,
                                                           const double* __restrict__ Wv, int emb,
                                                           const double* __restrict__ mix1w,
                                                           const double* __restrict__ mix1b,
                                                           const double* __restrict__ mix2w,
                                                           const double* __restrict__ mix2b, double* __restrict__ out) {
    extern __shared__ double Ms[];         // [16][n2max] scores
    __shared__ double red[16][16];
    const int b = blockIdx.x / n1max, i = blockIdx.x % n1max;
    const int h = threadIdx.x >> 4, l = threadIdx.x & 15;
    const double* crow = cost + (long)b * c_sb + (long)i * c_ld;
    double mloc = -__builtin_inf();
    for (int j = l; j < n2max; j += 16) {
        const double c = crow[j];
        double m = mix2b[h];
        for (int k = 0; k < 16; ++k) {
            // ms1 = 0 * mix1[h][0][k] + c * mix1[h][1][k] + mix1_bias[h][k]
            const double a = fma(c, mix1w[(h * 2 + 1) * 16 + k], mix1b[h * 16 + k]);
            m = fma(a > 0.0 ? a : 0.0, mix2w[h * 16 + k], m);
        }
        Ms[h * n2max + j] = m;
        mloc = fmax(mloc, m);
    }
    red[h][l] = mloc;
    __syncthreads();
    double mx = -__builtin_inf();
    for (int k = 0; k < 16; ++k) mx = fmax(mx, red[h][k]);
    __syncthreads();
    double sl = 0.0;
    for (int j = l; j < n2max; j += 16) sl += exp(Ms[h * n2max + j] - mx);
    red[h][l] = sl;
    __syncthreads();
    double sum = 0.0;
    for (int k = 0; k < 16; ++k) sum += red[h][k];
    const int n2b = n2[b];
    const double* wv = Wv + (long)(h * 16 + l) * emb;
    double acc = 0.0;
    for (int j = 0; j < n2b; ++j) acc = fma(exp(Ms[h * n2max + j] - mx), wv[j], acc);
    out[((long)b * n1max + i) * 256 + h * 16 + l] = acc / sum;
}

// C[m][n] = act(sum_k A[m][k] W[n][k] + bias[n]); 64 x 64 tiles, 256 threads of 4 x 4 outputs,
// K in steps of 16 through LDS.
__global__ __launch_bounds__(256) void gemm_f64_kernel(const double* __restrict__ A, int lda, const double* __restrict__ Wt,
                                                       int ldw, const double* __restrict__ bias, double* __restrict__ Cm,
                                                       int ldc, int M, int N, int K, int relu) {
    __shared__ double As[16][64 + 1], Ws[16][64 + 1];
    const int tid = threadIdx.x, tm = tid >> 4, tn = tid & 15;
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    double acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += 16) {
        for (int q = tid; q < 64 * 16; q += 256) {
            const int r = q >> 4, k = q & 15;
            const int gm = m0 + r, gn = n0 + r, gk = k0 + k;
            As[k][r] = (gm < M && gk < K) ? A[(long)gm * lda + gk] : 0.0;
            Ws[k][r] = (gn < N && gk < K) ? Wt[(long)gn * ldw + gk] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            double a[4], w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a[u] = As[k][tm * 4 + u];
                w[u] = Ws[k][tn * 4 + u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[u][v] = fma(a[u], w[v], acc[u][v]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int gm = m0 + tm * 4 + u;
        if (gm >= M) continue;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int gn = n0 + tn * 4 + v;
            if (gn >= N) continue;
            double y = acc[u][v] + (bias ? bias[gn] : 0.0);
            if (relu && y < 0.0) y = 0.0;
            Cm[(long)gm * ldc + gn] = y;
        }
    }
}

// InstanceNorm1d over the P positions of each pair and channel (afau.py:154-176, affine, biased
// variance, eps): x = in1 (+ in2), or (in1 NULL) the col block's one-hot + bias
// x[r][c] = [r < nvalid[b] and r == c] + obias[c].  out (optional) and gmax[b][c] = max_r y (optional).
// One thread per (pair, channel), two passes over the rows.
__global__ __launch_bounds__(64) void instnorm_f64_kernel(const double* __restrict__ in1, const double* __restrict__ in2,
                                                          int P, int Cn, const int* __restrict__ nvalid,
                                                          const double* __restrict__ obias, const double* __restrict__ w,
                                                          const double* __restrict__ bb, double eps,
                                                          double* __restrict__ out, double* __restrict__ gmax) {
    const int c = blockIdx.x * 64 + threadIdx.x, b = blockIdx.y;
    if (c >= Cn) return;
    const long base = (long)b * P * Cn + c;
    auto xv = [&](int r) -> double {
        if (!in1) return ((nvalid && r < nvalid[b] && r == c) ? 1.0 : 0.0) + obias[c];
        double v = in1[base + (long)r * Cn];
        if (in2) v += in2[base + (long)r * Cn];
        return v;
    };
    double mean = 0.0;
    for (int r = 0; r < P; ++r) mean += xv(r);
    mean /= (double)P;
    double var = 0.0;
    for (int r = 0; r < P; ++r) {
        const double t = xv(r) - mean;
        var = fma(t, t, var);
    }
    var /= (double)P;
    const double rs = 1.0 / sqrt(var + eps), sc = w[c], sh = bb[c];
    double mx = -__builtin_inf();
    for (int r = 0; r < P; ++r) {
        const double y = (xv(r) - mean) * rs * sc + sh;
        if (out) out[base + (long)r * Cn] = y;
        mx = fmax(mx, y);
    }
    if (gmax) gmax[(long)b * Cn + c] = mx;
}

// ks[b] = sigmoid((final_row(gr[b]) + final_col(gc[cidx[b]])) / 2), final_* = Linear(E, 8), ReLU,
// Linear(8, 1) (ngm.py:180-190, 401-412 with mean_k).  One workgroup of 64 per pair.
__global__ __launch_bounds__(64) void afau_head_f64_kernel(const double* __restrict__ gr, const double* __restrict__ gc,
                                                           const int* __restrict__ cidx, int E,
                                                           const double* __restrict__ r0w, const double* __restrict__ r0b,
                                                           const double* __restrict__ r2w, const double* __restrict__ r2b,
                                                           const double* __restrict__ c0w, const double* __restrict__ c0b,
                                                           const double* __restrict__ c2w, const double* __restrict__ c2b,
                                                           float* __restrict__ ks) {
    __shared__ double part[16][64];
    const int b = blockIdx.x, t = threadIdx.x;
    const double* g0 = gr + (long)b * E;
    const double* g1 = gc + (long)(cidx ? cidx[b] : b) * E;
    for (int u = 0; u < 8; ++u) {
        double a = 0.0, c = 0.0;
        for (int k = t; k < E; k += 64) {
            a = fma(r0w[(long)u * E + k], g0[k], a);
            c = fma(c0w[(long)u * E + k], g1[k], c);
        }
        part[u][t] = a;
        part[8 + u][t] = c;
    }
    __syncthreads();
    if (t != 0) return;
    double kr = r2b[0], kc = c2b[0];
    for (int u = 0; u < 8; ++u) {
        double a = r0b[u], c = c0b[u];
        for (int k = 0; k < 64; ++k) {
            a += part[u][k];
            c += part[8 + u][k];
        }
        kr = fma(r2w[u], a > 0.0 ? a : 0.0, kr);
        kc = fma(c2w[u], c > 0.0 ? c : 0.0, kc);
    }
    const double lg = 0.5 * (kr + kc);
    ks[b] = (float)(1.0 / (1.0 + exp(-lg)));
}

// soft_topk + Sinkhorn_m.forward_log (soft_topk.py:8-53, 166-255, batched_operation=False) in fp64:
// per pair the valid block's entries x_e (row-major, N = n1 n2) against the anchors [min, max] of the
// block, L[e][c] = -|x_e - anchor_c| / tau; alternately L -= logsumexp over the 2 columns (+ log 1,
// the row marginal) and L -= logsumexp over the N rows + log [N - k, k]; NaN -> -inf; ``iters`` steps,
// then further steps while any L > 0 (the reference's while loop; capped at PK_MAX_STEPS so every
// wave reaches the exit); ds[i][j] = exp(L[i n2 + j][1]) on the block, 0 elsewhere.  One workgroup
// per pair, L in a global fp64 scratch (2 N doubles per pair, L2-resident), block reductions.
constexpr int PK_MAX_STEPS = 100000;

// op 0: sum, 1: max, 2: min; every thread gets the result (fixed order: wave butterfly, then waves
// in order)
__device__ __forceinline__ double block_reduce(double v, int op, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 32; o > 0; o >>= 1) {
        const double y = __shfl_xor(v, o);
        v = op == 0 ? v + y : op == 1 ? fmax(v, y) : fmin(v, y);
    }
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double r = red[0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = op == 0 ? r + red[k] : op == 1 ? fmax(r, red[k]) : fmin(r, red[k]);
    return r;
}

__global__ __launch_bounds__(256) void soft_topk_f64_kernel(const double* __restrict__ ss, long s_sb, long s_ld,
                                                            const int* __restrict__ n1, const int* __restrict__ n2,
                                                            const float* __restrict__ kk, int n1max, int n2max,
                                                            int iters, double tau, double* __restrict__ ws,
                                                            float* __restrict__ out, long o_sb, long o_ld,
                                                            int* __restrict__ steps_out, float* __restrict__ out2,
                                                            long o2_sb, long o2_ld) {
    __shared__ double red[4];
    const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const int r = n1[b], c = n2[b];
    const long N = (long)r * c;
    const double NEG = -__builtin_inf();
    const double* sb = ss + (long)b * s_sb;
    double* L = ws + (long)b * 2 * n1max * n2max;
    int st = 0;
    if (N > 0) {
        double mn = __builtin_inf(), mx = NEG;
        for (long e = tid; e < N; e += nt) {
            const double v = sb[(e / c) * s_ld + e % c];
            mn = fmin(mn, v);
            mx = fmax(mx, v);
        }
        mn = block_reduce(mn, 2, red);
        mx = block_reduce(mx, 1, red);
        for (long e = tid; e < N; e += nt) {
            const double v = sb[(e / c) * s_ld + e % c];
            L[2 * e] = -fabs(v - mn) / tau;
            L[2 * e + 1] = -fabs(v - mx) / tau;
        }
        const double k = (double)kk[b];
        const double lcp[2] = {log((double)N - k), log(k)};
        auto fix = [&](double y) { return y != y ? NEG : y; };
        auto step = [&](int i) {
            __syncthreads();
            if ((i & 1) == 0) {
                for (long e = tid; e < N; e += nt) {
                    const double a = L[2 * e], q = L[2 * e + 1];
                    const double m = fmax(a, q);
                    const double lse = m == NEG ? NEG : m + log(exp(a - m) + exp(q - m));
                    L[2 * e] = fix(a - lse + 0.0);
                    L[2 * e + 1] = fix(q - lse + 0.0);
                }
            } else {
                double lse[2];
                for (int cc = 0; cc < 2; ++cc) {
                    double m = NEG;
                    for (long e = tid; e < N; e += nt) m = fmax(m, L[2 * e + cc]);
                    m = block_reduce(m, 1, red);
                    double sum = 0.0;
                    if (m != NEG)
                        for (long e = tid; e < N; e += nt) sum += exp(L[2 * e + cc] - m);
                    sum = block_reduce(sum, 0, red);
                    lse[cc] = m == NEG ? NEG : m + log(sum);
                }
                for (long e = tid; e < N; e += nt) {
                    L[2 * e] = fix(L[2 * e] - lse[0] + lcp[0]);
                    L[2 * e + 1] = fix(L[2 * e + 1] - lse[1] + lcp[1]);
                }
            }
        };
        for (; st < iters; ++st) step(st);
        for (;;) {
            __syncthreads();
            double pos = 0.0;
            for (long e = tid; e < 2 * N; e += nt) pos = fmax(pos, L[e] > 0.0 ? 1.0 : 0.0);
            pos = block_reduce(pos, 1, red);
            if (pos == 0.0 || st >= PK_MAX_STEPS) break;
            step(st);
            ++st;
        }
        __syncthreads();
    }
    for (long q = tid; q < (long)n1max * n2max; q += nt) {
        const int i = (int)(q / n2max), j = (int)(q % n2max);
        const float v = (i < r && j < c) ? (float)exp(L[2 * ((long)i * c + j) + 1]) : 0.f;
        out[(long)b * o_sb + (long)i * o_ld + j] = v;
        if (out2) out2[(long)b * o2_sb + (long)i * o2_ld + j] = v;
    }
    if (steps_out && tid == 0) steps_out[b] = st;
}

}  // namespace

extern "C" int fpm_soft_topk_fwd_f64(const double* ss, long s_sb, long s_ld, const int* n1, const int* n2,
                                     const float* k, int B, int n1max, int n2max, int iters, double tau, double* ws,
                                     long ws_doubles, float* out, long o_sb, long o_ld, int* steps_out, float* out2,
                                     long o2_sb, long o2_ld, void* stream) {
    if (B == 0) return 0;
    FPM_CHECK_ARG(n1max > 0 && n2max > 0 && iters >= 0 && tau > 0.0, "soft_topk_f64: bad sizes / iters / tau");
    FPM_CHECK_ARG(ws_doubles >= 2L * B * n1max * n2max, "soft_topk_f64: workspace of 2 B n1max n2max doubles needed");
    hipLaunchKernelGGL(soft_topk_f64_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, ss, s_sb, s_ld, n1, n2,
                       k, n1max, n2max, iters, tau, ws, out, o_sb, o_ld, steps_out, out2, o2_sb, o2_ld);
    return fpm::check_launch("fpm_soft_topk_fwd_f64");
}

extern "C" int fpm_kron_gnn_layer_fwd_f64(const void* X, int x_f64, int C, int B, int n1max, int n2max, const int* ptr1,
                                          const int* nbr1, const int* ptr2, const int* nbr2, const int* n1,
                                          const int* n2, const float* params, double* Xout, double* zbuf, void* stream) {
    FPM_CHECK_ARG(C == 1 || C == 17, "gnn_layer_f64: C must be 1 or 17 (got %d)", C);
    FPM_CHECK_ARG(x_f64 == (C == 17), "gnn_layer_f64: layer 0 (C = 1) reads fp32 Kp, later layers the fp64 state");
    if (B == 0) return 0;
    FPM_CHECK_ARG(n1max >= 1 && n1max <= 1024 && n2max >= 1, "gnn_layer_f64: n1max must be in [1, 1024]");
    const size_t sh = (size_t)C * n1max * 8;
    FPM_CHECK_ARG(sh <= 160 * 1024, "gnn_layer_f64: 17 x n1max doubles must fit LDS");
    const int threads = (n1max + 63) / 64 * 64;
    const unsigned grid = (unsigned)(((B + 7) / 8) * 8 * n2max);
    hipStream_t st = (hipStream_t)stream;
    if (C == 1) {
        auto k = gnn_layer_f64_kernel<1, float>;
        hipLaunchKernelGGL(k, dim3(grid), dim3(threads), sh, st, (const float*)X, n1max, n2max, ptr1, nbr1, ptr2,
                           nbr2, n1, n2, params, Xout, zbuf, B);
    } else {
        auto k = gnn_layer_f64_kernel<17, double>;
        if (sh > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        hipLaunchKernelGGL(k, dim3(grid), dim3(threads), sh, st, (const double*)X, n1max, n2max, ptr1, nbr1, ptr2,
                           nbr2, n1, n2, params, Xout, zbuf, B);
    }
    return fpm::check_launch("fpm_kron_gnn_layer_fwd_f64");
}

extern "C" int fpm_sinkhorn_log_fwd_f64(const void* s, int s_f64, long s_sb, long s_si, long s_sj, double* o64,
                                        long o_sb, long o_si, long o_sj, float* o32, long f_sb, long f_si, long f_sj,
                                        const int* n1, const int* n2, int B, int n1max, int n2max, int iters,
                                        double tau, int dummy_row, void* stream) {
    if (B == 0) return 0;
    FPM_CHECK_ARG(o64 || o32, "sinkhorn_f64: no output");
    FPM_CHECK_ARG(n1max >= 1 && n2max >= 1 && n1max <= 128 && n2max <= 128,
                  "sinkhorn_f64: the LDS-resident block holds boxes up to 128 x 128 (got %d x %d)", n1max, n2max);
    FPM_CHECK_ARG(tau > 0.0 && iters >= 0, "sinkhorn_f64: tau > 0 and iters >= 0");
    const int m = n1max > n2max ? n1max : n2max;
    const size_t sh = (size_t)m * (m + 1) * 8;
    hipStream_t st = (hipStream_t)stream;
    if (s_f64) {
        auto k = sinkhorn_f64_kernel<double>;
        if (sh > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        hipLaunchKernelGGL(k, dim3(B), dim3(256), sh, st, (const double*)s, s_sb, s_si, s_sj, o64, o_sb, o_si, o_sj,
                           o32, f_sb, f_si, f_sj, n1, n2, n1max, n2max, iters, tau, dummy_row);
    } else {
        auto k = sinkhorn_f64_kernel<float>;
        if (sh > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        hipLaunchKernelGGL(k, dim3(B), dim3(256), sh, st, (const float*)s, s_sb, s_si, s_sj, o64, o_sb, o_si, o_sj,
                           o32, f_sb, f_si, f_sj, n1, n2, n1max, n2max, iters, tau, dummy_row);
    }
    return fpm::check_launch("fpm_sinkhorn_log_fwd_f64");
}

extern "C" int fpm_node_classifier_f64(const double* X, int B, int n1max, int n2max, const float* w, const float* bias,
                                       double* s64, float* s32, void* stream) {
    if (B == 0) return 0;
    const long total = (long)B * n1max * n2max;
    FPM_CHECK_ARG(total < (1L << 31) * 256L, "node_classifier_f64: batch too large");
    hipLaunchKernelGGL(classifier_f64_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       X, n1max, n2max, w, bias, s64, s32, B);
    return fpm::check_launch("fpm_node_classifier_f64");
}

extern "C" int fpm_crossset_attn_row_f64(const double* cost, long c_sb, long c_ld, int B, int n1max, int n2max,
                                         const int* n2, const double* Wv, int emb, const double* mix1w,
                                         const double* mix1b, const double* mix2w, const double* mix2b, double* out,
                                         void* stream) {
    if (B == 0 || n1max == 0) return 0;
    FPM_CHECK_ARG(n2max >= 1 && n2max <= emb, "crossset_attn_row_f64: 1 <= n2max <= emb (UNIV_SIZE)");
    const size_t sh = (size_t)16 * n2max * 8;
    FPM_CHECK_ARG(sh <= 96 * 1024, "crossset_attn_row_f64: n2max too large");
    if (sh > 65536)
        (void)hipFuncSetAttribute((const void*)attn_row_f64_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    hipLaunchKernelGGL(attn_row_f64_kernel, dim3((unsigned)(B * n1max)), dim3(256), sh, (hipStream_t)stream, cost, c_sb,
                       c_ld, n1max, n2max, n2, Wv, emb, mix1w, mix1b, mix2w, mix2b, out);
    return fpm::check_launch("fpm_crossset_attn_row_f64");
}

extern "C" int fpm_gemm_f64(const double* A, int lda, const double* W, int ldw, const double* bias, double* C, int ldc,
                            int M, int N, int K, int relu, void* stream) {
    if (M == 0 || N == 0) return 0;
    FPM_CHECK_ARG(lda >= K && ldw >= K && ldc >= N && K >= 0, "gemm_f64: leading dimensions");
    FPM_CHECK_ARG(M <= 65535 * 64, "gemm_f64: M too large");
    const dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64));
    hipLaunchKernelGGL(gemm_f64_kernel, grid, dim3(256), 0, (hipStream_t)stream, A, lda, W, ldw, bias, C, ldc, M, N, K,
                       relu);
    return fpm::check_launch("fpm_gemm_f64");
}

extern "C" int fpm_instnorm_f64(const double* in1, const double* in2, int B, int P, int Cn, const int* nvalid,
                                const double* onehot_bias, const double* w, const double* bias, double eps, double* out,
                                double* gmax, void* stream) {
    if (B == 0) return 0;
    FPM_CHECK_ARG(P >= 1 && Cn >= 1 && B <= 65535, "instnorm_f64: P, Cn >= 1, B <= 65535");
    FPM_CHECK_ARG(in1 || onehot_bias, "instnorm_f64: in1 or onehot_bias");
    FPM_CHECK_ARG(out || gmax, "instnorm_f64: no output");
    hipLaunchKernelGGL(instnorm_f64_kernel, dim3((unsigned)((Cn + 63) / 64), (unsigned)B), dim3(64), 0,
                       (hipStream_t)stream, in1, in2, P, Cn, nvalid, onehot_bias, w, bias, eps, out, gmax);
    return fpm::check_launch("fpm_instnorm_f64");
}

extern "C" int fpm_afau_head_f64(const double* gr, const double* gc, const int* cidx, int B, int E, const double* r0w,
                                 const double* r0b, const double* r2w, const double* r2b, const double* c0w,
                                 const double* c0b, const double* c2w, const double* c2b, float* ks, void* stream) {
    if (B == 0) return 0;
    hipLaunchKernelGGL(afau_head_f64_kernel, dim3((unsigned)B), dim3(64), 0, (hipStream_t)stream, gr, gc, cidx, E, r0w,
                       r0b, r2w, r2b, c0w, c0b, c2w, c2b, ks);
    return fpm::check_launch("fpm_afau_head_f64");
}
