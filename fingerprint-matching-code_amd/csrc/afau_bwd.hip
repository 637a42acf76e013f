// Backward of the AFA-U k regressor (reference src/model/afau.py:54-300 and ngm.py:386-412, as
// trained by training_loop.py:23-70 through ks_loss; ss is detached at ngm.py:398, so nothing
// flows back into the matcher).  The forward is the HIP one (afau.hip) in fp32, with its
// intermediates kept; these kernels run the reverse pass:
//   head:       ks = sigmoid((final_row(gr) + final_col(gc)) / 2)       -> dgr, dgc, head grads
//   max pool:   gr = max over positions of r                           -> one-hot seed per channel
//   instnorm:   y = (x - mean) rstd w + b over positions (afau.py:154-176) -> dx, dw, db
//   attention:  out_h(i) = sum_j softmax_j(f_h(cost_ij)) Wv[h*16:, j]  -> dWv, mixed-score grads
// (with R0 = 0 the query, the key and the dot-product input of the mixed score are identically 0,
// so Wq, Wk and mix1_weight[:, 0] have exactly zero gradient; the col block's attention output is
// 0 and its combine bias is cancelled by the instance norm).  The FFN / combine products are the
// MFMA GEMMs of fpm_gemm on transposed operands (fpm_transpose), split over K where K = rows.
// Per-pair partial sums are reduced over pairs in a fixed order (fpm_rows_sum), so the gradients
// are deterministic.
#include "fpm_common.h"

namespace {

// ---- head: per pair, both 600 -> 8 -> 1 heads; per-pair parameter-gradient partials
//   part[b] = [dW0r (8 x E) | db0r (8) | dw2r (8) | db2r | dW0c (8 x E) | db0c (8) | dw2c (8) | db2c]
__global__ __launch_bounds__(256) void afau_head_bwd_kernel(const float* __restrict__ gr, const float* __restrict__ gc,
                                                            int E, const float* __restrict__ r0w,
                                                            const float* __restrict__ r0b,
                                                            const float* __restrict__ r2w,
                                                            const float* __restrict__ r2b,
                                                            const float* __restrict__ c0w,
                                                            const float* __restrict__ c0b,
                                                            const float* __restrict__ c2w,
                                                            const float* __restrict__ c2b,
                                                            const float* __restrict__ dks, float* __restrict__ dgr,
                                                            float* __restrict__ dgc, float* __restrict__ part) {
    __shared__ float hid[2][8], red[2][8][4];
    __shared__ float g2[2][8], dk_s;
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const float* G[2] = {gr + (long)b * E, gc + (long)b * E};
    const float* W0[2] = {r0w, c0w};
    const float* B0[2] = {r0b, c0b};
    const float* W2[2] = {r2w, c2w};
    const float* B2[2] = {r2b, c2b};
    // hidden pre-activations: 16 dot products of length E, 4 waves each over a quarter
    for (int q = 0; q < 2; ++q)
        for (int m = 0; m < 8; ++m) {
            float s = 0.f;
            for (int c = tid; c < E; c += 256) s = fmaf(W0[q][m * E + c], G[q][c], s);
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
            if (lane == 0) red[q][m][wv] = s;
        }
    __syncthreads();
    if (tid < 16) {
        const int q = tid >> 3, m = tid & 7;
        hid[q][m] = red[q][m][0] + red[q][m][1] + red[q][m][2] + red[q][m][3] + B0[q][m];
    }
    __syncthreads();
    if (tid == 0) {
        float k[2];
        for (int q = 0; q < 2; ++q) {
            float s = B2[q][0];
            for (int m = 0; m < 8; ++m) s = fmaf(W2[q][m], fmaxf(hid[q][m], 0.f), s);
            k[q] = s;
        }
        const float ks = 1.f / (1.f + expf(-((k[0] + k[1]) / 2.f)));
        dk_s = dks[b] * ks * (1.f - ks) * 0.5f;        // d(kr) = d(kc)
    }
    __syncthreads();
    const float dk = dk_s;
    if (tid < 16) {
        const int q = tid >> 3, m = tid & 7;
        g2[q][m] = hid[q][m] > 0.f ? dk * W2[q][m] : 0.f;
    }
    __syncthreads();
    const long PS = 8L * E + 17;                           // one head's partial block
    float* pb = part + (long)b * 2 * PS;
    for (int q = 0; q < 2; ++q) {
        float* dg = (q == 0 ? dgr : dgc) + (long)b * E;
        for (int c = tid; c < E; c += 256) {
            float s = 0.f;
            for (int m = 0; m < 8; ++m) {
                s = fmaf(W0[q][m * E + c], g2[q][m], s);
                pb[q * PS + m * E + c] = g2[q][m] * G[q][c];
            }
            dg[c] = s;
        }
        if (tid < 8) {
            pb[q * PS + 8L * E + tid] = g2[q][tid];
            pb[q * PS + 8L * E + 8 + tid] = dk * fmaxf(hid[q][tid], 0.f);
        }
        if (tid == 0) pb[q * PS + 8L * E + 16] = dk;
    }
}

// ---- instance-norm backward over positions, per (pair, 64-channel tile): 16 position groups x
// 64 channels, the <= NV positions of a thread in registers.  Input x = in1 (+ in2), or the col
// block's synthesised one-hot + bias.  Seed: dense dy, or (gseed != null) the max pool's gradient
// gseed[b][c] routed to the first position holding the max of y.
template <int NV>
__global__ __launch_bounds__(1024) void instnorm_bwd_kernel(const float* __restrict__ in1, const float* __restrict__ in2,
                                                            int P, int Cn, const int* __restrict__ nvalid,
                                                            const float* __restrict__ onehot_bias,
                                                            const float* __restrict__ w, const float* __restrict__ bb,
                                                            float eps, const float* __restrict__ dy,
                                                            const float* __restrict__ gseed, float* __restrict__ dx,
                                                            int accumulate, float* __restrict__ dw_part,
                                                            float* __restrict__ db_part) {
    __shared__ float red[16][64];
    __shared__ float red2[16][64];
    __shared__ int redp[16][64];
    const int b = blockIdx.x, cl = threadIdx.x & 63, c = blockIdx.y * 64 + cl, g = threadIdx.x >> 6;
    const bool cv = c < Cn;
    const int nb = onehot_bias ? nvalid[b] : 0;
    float v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int p = g + 16 * k;
        float x = 0.f;
        if (cv && p < P) {
            if (onehot_bias) {
                x = ((p == c && p < nb) ? 1.f : 0.f) + onehot_bias[c];
            } else {
                const long o = ((long)b * P + p) * Cn + c;
                x = in2 ? in1[o] + in2[o] : in1[o];
            }
        }
        v[k] = x;
    }
    // statistics exactly as the forward computes them (same order, same values)
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) s += v[k];
    red[g][cl] = s;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) tot += red[q][cl];
    const float mean = tot / (float)P;
    __syncthreads();
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int p = g + 16 * k;
        const float d = v[k] - mean;
        if (p < P) sq += d * d;
    }
    red[g][cl] = sq;
    __syncthreads();
    float var = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) var += red[q][cl];
    var /= (float)P;
    const float rstd = 1.f / sqrtf(var + eps);
    const float ww = cv ? w[c] : 0.f, bv = cv ? bb[c] : 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = (v[k] - mean) * rstd;          // xhat
    float g_at[NV];
    if (gseed) {
        // argmax over positions of y = xhat w + b; ties -> the smallest position
        float mx = -INFINITY;
        int pm = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int p = g + 16 * k;
            if (!cv || p >= P) continue;
            const float y = v[k] * ww + bv;
            if (y > mx) { mx = y; pm = p; }
        }
        __syncthreads();
        red[g][cl] = mx;
        redp[g][cl] = pm;
        __syncthreads();
        float M = red[0][cl];
        int PM = redp[0][cl];
        for (int q = 1; q < 16; ++q) {
            const float m2 = red[q][cl];
            const int p2 = redp[q][cl];
            if (m2 > M || (m2 == M && p2 < PM)) { M = m2; PM = p2; }
        }
        const float gs = cv ? gseed[(long)b * Cn + c] : 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) g_at[k] = (g + 16 * k == PM) ? gs : 0.f;
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int p = g + 16 * k;
            g_at[k] = (cv && p < P) ? dy[((long)b * P + p) * Cn + c] : 0.f;
        }
    }
    // dxhat = dy w;  dx = rstd (dxhat - mean(dxhat) - xhat mean(dxhat xhat))
    float s1 = 0.f, s2 = 0.f, sw = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const float dxh = g_at[k] * ww;
        s1 += dxh;
        s2 += dxh * v[k];
        sw += g_at[k] * v[k];
        sb += g_at[k];
    }
    __syncthreads();
    red[g][cl] = s1;
    red2[g][cl] = s2;
    __syncthreads();
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        t1 += red[q][cl];
        t2 += red2[q][cl];
    }
    const float m1 = t1 / (float)P, m2 = t2 / (float)P;
    if (dx) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int p = g + 16 * k;
            if (!cv || p >= P) continue;
            const long o = ((long)b * P + p) * Cn + c;
            const float d = rstd * (g_at[k] * ww - m1 - v[k] * m2);
            dx[o] = accumulate ? dx[o] + d : d;
        }
    }
    __syncthreads();
    red[g][cl] = sw;
    red2[g][cl] = sb;
    __syncthreads();
    if (g == 0 && cv) {
        float a = 0.f, e = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            a += red[q][cl];
            e += red2[q][cl];
        }
        dw_part[(long)b * Cn + c] = a;
        db_part[(long)b * Cn + c] = e;
    }
}

// ---- row-block attention backward: one workgroup per (pair, head), thread t owns the columns
// j = t + 256 u (u < TJ); rows i are walked in order.  Per (i, j):
//   score = f_h(cost_ij) (16-term sum), att = exp(score - M_i) / S_i (forward statistics),
//   dA = datt_h(i) . v_h(j),  dscore = att (dA - datt_h(i) . out_h(i)),
//   dWv[h*16 + d][j] += att datt_h(i)[d]  (j < n2b; v = 0 beyond),
//   mixed-score grads through the active hidden units (pre = w1 c + b1 > 0).
// Outputs per pair: dwv_part[b][h*16 + d][j] (j < n2max) and mix_part[b][h][49] =
// [dW2 (16) | dW1 row 1 (16) | db1 (16) | db2].
template <int TJ>
__global__ __launch_bounds__(256) void afau_attn_bwd_kernel(const float* __restrict__ cost, long c_sb, long c_ld,
                                                            int n1max, int n2max, const int* __restrict__ n2,
                                                            const float* __restrict__ Wv, int emb,
                                                            const float* __restrict__ mix1w,
                                                            const float* __restrict__ mix1b,
                                                            const float* __restrict__ mix2w,
                                                            const float* __restrict__ mix2b,
                                                            const float* __restrict__ att_out,
                                                            const float* __restrict__ datt,
                                                            const float2* __restrict__ stats,
                                                            float* __restrict__ dwv_part,
                                                            float* __restrict__ mix_part) {
    __shared__ float red[49][4];
    const int b = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n2b = n2[b];
    float w1[16], b1[16], w2[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        w1[m] = mix1w[(h * 2 + 1) * 16 + m];
        b1[m] = mix1b[h * 16 + m];
        w2[m] = mix2w[h * 16 + m];
    }
    const float b2 = mix2b[h];
    float vj[TJ][16], dwv[TJ][16];
#pragma unroll
    for (int u = 0; u < TJ; ++u) {
        const int j = tid + 256 * u;
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            vj[u][d] = j < n2b ? Wv[(long)(h * 16 + d) * emb + j] : 0.f;
            dwv[u][d] = 0.f;
        }
    }
    // gb1 is a bias-like sum: sum_j ds_ij = 0 in every row (softmax), so sum over the active entries
    // = -(sum over the inactive ones); both are accumulated and the one over fewer entries is used
    // (a unit active on all of [0, 1] then gets its exact gradient 0 instead of cancellation noise).
    // mix2_bias shifts every score of a head: its gradient is exactly 0 (gb2 is not accumulated).
    float gw2[16], gw1[16], gb1[16], gb1n[16];
    int nact[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        gw2[m] = gw1[m] = gb1[m] = gb1n[m] = 0.f;
        nact[m] = 0;
    }
    int ntot = 0;
    const float* Cb = cost + (long)b * c_sb;
    __shared__ float dred[2][4];
    for (int i = 0; i < n1max; ++i) {
        const long row = (long)b * n1max + i;
        float da[16];
#pragma unroll
        for (int d = 0; d < 16; ++d) da[d] = datt[row * 256 + h * 16 + d];
        const float2 st = stats[row * 16 + h];
        const float invS = 1.f / st.y;
        float cj[TJ], att[TJ], dA[TJ];
        float part = 0.f;
#pragma unroll
        for (int u = 0; u < TJ; ++u) {
            const int j = tid + 256 * u;
            cj[u] = 0.f;
            att[u] = 0.f;
            dA[u] = 0.f;
            if (j >= n2max) continue;
            const float c = Cb[(long)i * c_ld + j];
            float sc = 0.f;
#pragma unroll
            for (int m = 0; m < 16; ++m) sc += fmaxf(c * w1[m] + b1[m], 0.f) * w2[m];
            sc += b2;
            cj[u] = c;
            att[u] = expf(sc - st.x) * invS;
            float a = 0.f;
#pragma unroll
            for (int d = 0; d < 16; ++d) a = fmaf(da[d], vj[u][d], a);
            dA[u] = a;
            part = fmaf(att[u], a, part);
        }
        // the softmax backward's row term sum_j att dA, reduced exactly over the row (not taken
        // as datt . out from the forward: the bias-like parameters' true gradient is a sum with
        // heavy cancellation, which a 1-ulp mismatch between the two would bias)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
        if (lane == 0) dred[i & 1][wv] = part;
        __syncthreads();
        const float dot = ((dred[i & 1][0] + dred[i & 1][1]) + dred[i & 1][2]) + dred[i & 1][3];
#pragma unroll
        for (int u = 0; u < TJ; ++u) {
            const int j = tid + 256 * u;
            if (j >= n2max) continue;
            const float c = cj[u];
#pragma unroll
            for (int d = 0; d < 16; ++d) dwv[u][d] = fmaf(att[u], da[d], dwv[u][d]);
            const float ds = att[u] * (dA[u] - dot);
            ++ntot;
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const float pre = c * w1[m] + b1[m];
                if (pre > 0.f) {
                    gw2[m] = fmaf(ds, pre, gw2[m]);
                    const float t = ds * w2[m];
                    gw1[m] = fmaf(t, c, gw1[m]);
                    gb1[m] += t;
                    ++nact[m];
                } else {
                    gb1n[m] = fmaf(ds, w2[m], gb1n[m]);
                }
            }
        }
    }
#pragma unroll
    for (int u = 0; u < TJ; ++u) {
        const int j = tid + 256 * u;
        if (j >= n2max) continue;
#pragma unroll
        for (int d = 0; d < 16; ++d)
            dwv_part[((long)b * 256 + h * 16 + d) * n2max + j] = j < n2b ? dwv[u][d] : 0.f;
    }
    // workgroup reduction of the 49 mixed-score partials: waves, then the 4 wave sums in order
    auto wsum = [&](float x) {
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        return x;
    };
    auto isum = [&](int x) {
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        return x;
    };
    __shared__ float redn[16][4];
    __shared__ int cnt[17][4];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const float a = wsum(gw2[m]), e = wsum(gw1[m]), f = wsum(gb1[m]), fn = wsum(gb1n[m]);
        const int na = isum(nact[m]);
        if (lane == 0) {
            red[m][wv] = a;
            red[16 + m][wv] = e;
            red[32 + m][wv] = f;
            redn[m][wv] = fn;
            cnt[m][wv] = na;
        }
    }
    const int nt = isum(ntot);
    if (lane == 0) cnt[16][wv] = nt;
    __syncthreads();
    float* mp = mix_part + ((long)b * 16 + h) * 49;
    if (tid < 48) {
        float v = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
        if (tid >= 32) {
            const int m = tid - 32;
            const int na = cnt[m][0] + cnt[m][1] + cnt[m][2] + cnt[m][3];
            const int nn = cnt[16][0] + cnt[16][1] + cnt[16][2] + cnt[16][3] - na;
            if (nn < na) v = -(redn[m][0] + redn[m][1] + redn[m][2] + redn[m][3]);
        }
        mp[tid] = v;
    }
    if (tid == 48) mp[48] = 0.f;
}

// out[u][k] (+)= sum of in[b][k] over b in order: with key, the b with key[b] == u; without, the
// u-th of nkeys contiguous chunks of ceil(B / nkeys) rows (a two-level sum of many rows).  V = 4:
// four consecutive k per thread on 16-B loads / stores (K % 4 == 0, 16-B aligned rows); the keyless
// row loop is unrolled by 8 so eight row loads are in flight ahead of the in-order adds.  Every
// element's additions are the same, in the same order, for V = 1 and V = 4.
template <int V>
__global__ void rows_sum_kernel(const float* __restrict__ in, int B, long K, const int* __restrict__ key, int nkeys,
                                float* __restrict__ out, int accumulate) {
    typedef float vec __attribute__((ext_vector_type(V)));
    const long k = ((long)blockIdx.x * blockDim.x + threadIdx.x) * V;
    const int u = blockIdx.y;
    if (k >= K) return;
    vec s = (vec)0.f;
    if (key) {
        for (int b = 0; b < B; ++b)
            if (key[b] == u) s += *(const vec*)(in + (long)b * K + k);
    } else {
        const int cs = (B + nkeys - 1) / nkeys, b1 = min(B, (u + 1) * cs);
#pragma unroll 8
        for (int b = u * cs; b < b1; ++b) s += *(const vec*)(in + (long)b * K + k);
    }
    vec* o = (vec*)(out + (long)u * K + k);
    *o = accumulate ? *o + s : s;
}

// out[c][r] = in[r][c] (R x C -> C x ldo, columns [R, ldo) zero); 32 x 32 LDS tiles
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ in, long R, int C, long ldi,
                                                        float* __restrict__ out, long ldo) {
    __shared__ float t[32][33];
    const long r0 = (long)blockIdx.x * 32;
    const int c0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int k = ty; k < 32; k += 8) {
        const long r = r0 + k;
        const int c = c0 + tx;
        t[k][tx] = (r < R && c < C) ? in[r * ldi + c] : 0.f;
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        const int c = c0 + k;
        const long r = r0 + tx;
        if (c < C && r < ldo) out[(long)c * ldo + r] = t[tx][k];
    }
}

// elementwise: mode 0: x[i] = (ref[i] > 0) ? x[i] : 0 (ReLU backward through the post-activation);
// mode 1: x[i] += ref[i]
__global__ void ew_kernel(float* __restrict__ x, const float* __restrict__ ref, long n, int mode) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        if (mode == 0) x[i] = ref[i] > 0.f ? x[i] : 0.f;
        else x[i] += ref[i];
    }
}

}  // namespace

extern "C" int fpm_afau_head_bwd(const float* gr, const float* gc, int B, int E, const float* r0w, const float* r0b,
                                 const float* r2w, const float* r2b, const float* c0w, const float* c0b,
                                 const float* c2w, const float* c2b, const float* dks, float* dgr, float* dgc,
                                 float* part, void* stream) {
    FPM_CHECK_ARG(B >= 0 && E > 0, "afau_head_bwd: bad sizes");
    if (B == 0) return 0;
    hipLaunchKernelGGL(afau_head_bwd_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, gr, gc, E, r0w, r0b, r2w, r2b,
                       c0w, c0b, c2w, c2b, dks, dgr, dgc, part);
    return fpm::check_launch("fpm_afau_head_bwd");
}

extern "C" int fpm_instnorm_bwd(const float* in1, const float* in2, int B, int P, int Cn, const int* nvalid,
                                const float* onehot_bias, const float* w, const float* bias, float eps, const float* dy,
                                const float* gseed, float* dx, int accumulate, float* dw_part, float* db_part,
                                void* stream) {
    FPM_CHECK_ARG(B >= 0 && P > 0 && P <= 640 && Cn > 0, "instnorm_bwd: 0 < P <= 640 required");
    FPM_CHECK_ARG((dy != nullptr) != (gseed != nullptr), "instnorm_bwd: exactly one of dy / gseed");
    FPM_CHECK_ARG(onehot_bias ? nvalid != nullptr : in1 != nullptr, "instnorm_bwd: input missing");
    if (B == 0) return 0;
    dim3 grid(B, (Cn + 63) / 64);
    hipStream_t st = (hipStream_t)stream;
    if (P <= 256)
        hipLaunchKernelGGL((instnorm_bwd_kernel<16>), grid, dim3(1024), 0, st, in1, in2, P, Cn, nvalid, onehot_bias, w,
                           bias, eps, dy, gseed, dx, accumulate, dw_part, db_part);
    else
        hipLaunchKernelGGL((instnorm_bwd_kernel<40>), grid, dim3(1024), 0, st, in1, in2, P, Cn, nvalid, onehot_bias, w,
                           bias, eps, dy, gseed, dx, accumulate, dw_part, db_part);
    return fpm::check_launch("fpm_instnorm_bwd");
}

extern "C" int fpm_afau_attn_bwd(const float* cost, long c_sb, long c_ld, int B, int n1max, int n2max, const int* n2,
                                 const float* Wv, int emb, const float* mix1w, const float* mix1b, const float* mix2w,
                                 const float* mix2b, const float* att_out, const float* datt, const float* stats,
                                 float* dwv_part, float* mix_part, void* stream) {
    FPM_CHECK_ARG(B >= 0 && n1max > 0 && n2max > 0 && n2max <= 768 && n2max <= emb,
                  "afau_attn_bwd: 0 < n2max <= min(768, emb) required");
    if (B == 0) return 0;
    dim3 grid(B, 16);
    hipStream_t st = (hipStream_t)stream;
#define FPM_AB(TJ_)                                                                                              \
    hipLaunchKernelGGL((afau_attn_bwd_kernel<TJ_>), grid, dim3(256), 0, st, cost, c_sb, c_ld, n1max, n2max, n2, Wv, \
                       emb, mix1w, mix1b, mix2w, mix2b, att_out, datt, (const float2*)stats, dwv_part, mix_part)
    if (n2max <= 256) FPM_AB(1);
    else if (n2max <= 512) FPM_AB(2);
    else FPM_AB(3);
#undef FPM_AB
    return fpm::check_launch("fpm_afau_attn_bwd");
}

extern "C" int fpm_rows_sum(const float* in, int B, long K, const int* key, int nkeys, float* out, int accumulate,
                            void* stream) {
    FPM_CHECK_ARG(B >= 0 && K >= 0 && nkeys > 0, "rows_sum: bad sizes");
    if (K == 0) return 0;
    const bool v4 = K % 4 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0;
    if (v4) {
        dim3 grid((unsigned)((K / 4 + 255) / 256), nkeys);
        hipLaunchKernelGGL(rows_sum_kernel<4>, grid, dim3(256), 0, (hipStream_t)stream, in, B, K, key, nkeys, out,
                           accumulate);
    } else {
        dim3 grid((unsigned)((K + 255) / 256), nkeys);
        hipLaunchKernelGGL(rows_sum_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, in, B, K, key, nkeys, out,
                           accumulate);
    }
    return fpm::check_launch("fpm_rows_sum");
}

extern "C" int fpm_transpose(const float* in, long R, int C, long ldi, float* out, long ldo, void* stream) {
    FPM_CHECK_ARG(R >= 0 && C > 0 && ldi >= C && ldo >= R, "transpose: bad sizes");
    if (R == 0) return 0;
    dim3 grid((unsigned)((ldo + 31) / 32), (C + 31) / 32);
    hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, in, R, C, ldi, out, ldo);
    return fpm::check_launch("fpm_transpose");
}

extern "C" int fpm_elementwise(float* x, const float* ref, long n, int mode, void* stream) {
    FPM_CHECK_ARG(mode == 0 || mode == 1, "elementwise: mode 0 (relu mask) or 1 (add)");
    if (n <= 0) return 0;
    long blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(ew_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, ref, n, mode);
    return fpm::check_launch("fpm_elementwise");
}
