// AFA-U k regressor (reference ngm.py:386-412 over src/model/afau.py:54-300).
//
// With the reference's inputs R0 = 0 and C0 = one-hot (ngm.py:392-399):
//   row block: q = Wq R0 = 0, so the mixed score depends on the cost only:
//     score_h[i,j] = mix2_h . relu(mix1_h[1] * cost[i,j] + mix1_bias_h) + mix2_bias_h
//     out[i, h*16+d] = sum_j softmax_j(score_h[i,:]) * Wv[h*16+d, j]   (v = Wv C0, zero for j >= n2b)
//   col block: v = Wv R0 = 0, so the attention output is exactly 0 and o1 = IN(C0 + combine.bias).
// Kernels: the row-block cross-set attention, instance norm (optionally + residual, optionally
// fused with the max-pool over positions), and the 600->8->1 heads + sigmoid.
// The projections/FFN are MFMA GEMMs through fpm_gemm.
#include "fpm_common.h"

namespace {

// one workgroup per (pair, 16-row tile); 4 waves x 4 rows; heads looped.  The tile's costs stay
// in registers across the 16 heads (lane j-slots: j = lane + 64 jj, jj < NJ); scores stay in
// registers through max / exp / sum, and only the normalised probabilities go to LDS for AV.
template <typename T, int NJ>
__global__ __launch_bounds__(256) void afau_row_attn_kernel(const float* __restrict__ cost, long c_sb, long c_ld,
                                                            int n1max, int n2max, const int* __restrict__ n2,
                                                            const float* __restrict__ Wv, int emb,
                                                            const float* __restrict__ mix1w,
                                                            const float* __restrict__ mix1b,
                                                            const float* __restrict__ mix2w,
                                                            const float* __restrict__ mix2b, T* __restrict__ out) {
    constexpr int VS = 20;                // V row stride (floats): float4-aligned, spreads the LDS banks
    extern __shared__ float sh[];
    float* V = sh;                        // [n2max][VS]
    float* Pm = sh + n2max * VS;          // [16 rows][n2max]
    const int b = blockIdx.x, i0 = blockIdx.y * 16, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n2b = n2[b];
    const float* Cb = cost + (long)b * c_sb;
    float creg[4][NJ];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        const int i = i0 + wv * 4 + rr;
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
            const int j = lane + 64 * jj;
            creg[rr][jj] = (i < n1max && j < n2max) ? Cb[(long)i * c_ld + j] : 0.f;
        }
    }
    for (int h = 0; h < 16; ++h) {
        __syncthreads();
        for (int k = tid; k < n2max * 16; k += 256) {      // coalesced along j
            const int dd = k / n2max, j = k - dd * n2max;
            V[j * VS + dd] = j < n2b ? Wv[(long)(h * 16 + dd) * emb + j] : 0.f;
        }
        float w1[16], b1[16], w2[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            w1[m] = mix1w[(h * 2 + 1) * 16 + m];
            b1[m] = mix1b[h * 16 + m];
            w2[m] = mix2w[h * 16 + m];
        }
        const float b2 = mix2b[h];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int lr = wv * 4 + rr, i = i0 + lr;
            if (i >= n1max) break;
            float sv[NJ];
            float mx = -INFINITY;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                const float c = creg[rr][jj];
                float sc = 0.f;
#pragma unroll
                for (int m = 0; m < 16; ++m) sc += fmaxf(c * w1[m] + b1[m], 0.f) * w2[m];
                sc += b2;
                sv[jj] = sc;
                if (lane + 64 * jj < n2max) mx = fmaxf(mx, sc);
            }
            mx = fpm::warp_max(mx);
            float sum = 0.f;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                const float e = fpm::fast_exp2((sv[jj] - mx) * fpm::LOG2E_F);
                sv[jj] = e;
                if (lane + 64 * jj < n2max) sum += e;
            }
            sum = fpm::warp_sum(sum);
            const float inv = 1.f / sum;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                const int j = lane + 64 * jj;
                if (j < n2max) Pm[lr * n2max + j] = sv[jj] * inv;
            }
        }
        __syncthreads();
        // out[i][h*16 + d] for the 16 rows: thread = (row, 4 d's, j residue mod 4), float4 V reads
        {
            const int lr = tid >> 4, dq = (tid >> 2) & 3, jp = tid & 3, i = i0 + lr;
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int j = jp; j < n2max; j += 4) {
                const float pj = Pm[lr * n2max + j];
                const float4 v = *(const float4*)(V + j * VS + dq * 4);
                acc.x = fmaf(pj, v.x, acc.x);
                acc.y = fmaf(pj, v.y, acc.y);
                acc.z = fmaf(pj, v.z, acc.z);
                acc.w = fmaf(pj, v.w, acc.w);
            }
#pragma unroll
            for (int o = 1; o <= 2; o <<= 1) {
                acc.x += __shfl_xor(acc.x, o);
                acc.y += __shfl_xor(acc.y, o);
                acc.z += __shfl_xor(acc.z, o);
                acc.w += __shfl_xor(acc.w, o);
            }
            if (i < n1max && jp == 0) {
                T* o = out + ((long)b * n1max + i) * 256 + h * 16 + dq * 4;
                o[0] = fpm::from_f<T>(acc.x);
                o[1] = fpm::from_f<T>(acc.y);
                o[2] = fpm::from_f<T>(acc.z);
                o[3] = fpm::from_f<T>(acc.w);
            }
        }
    }
}

// InstanceNorm1d over positions (afau.py:145-176) of x = in1 (+ in2), or of the synthesised col
// input C0 + bias (onehot mode).  Writes out_f / out_t, or (gmax != null) only the max over
// positions of the normalised values (MaxPool1d over the -inf padded 600 positions, ngm.py:402-405).
// 1024 threads = 16 position groups x 64 channels; each thread keeps its <= NV values in registers,
// so x is read once (mean, variance and output from registers).
template <typename T, int NV>
__global__ __launch_bounds__(1024) void instnorm_kernel(const float* __restrict__ in1, const float* __restrict__ in2,
                                                        int P, int Cn, const int* __restrict__ nvalid,
                                                        const float* __restrict__ onehot_bias, const float* __restrict__ w,
                                                        const float* __restrict__ bb, float eps, float* __restrict__ out_f,
                                                        T* __restrict__ out_t, int ldt, float* __restrict__ gmax) {
    __shared__ float red[16][64];
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
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int p = g + 16 * k;
        if (!cv || p >= P) continue;
        const float y = (v[k] - mean) * rstd * ww + bv;
        if (gmax) mx = fmaxf(mx, y);
        else {
            const long o = ((long)b * P + p) * Cn + c;
            if (out_f) out_f[o] = y;
            if (out_t) out_t[((long)b * P + p) * ldt + c] = fpm::from_f<T>(y);
        }
    }
    // zero K-padding columns [Cn, ldt) of the operand copy (the next GEMM runs K = ldt)
    if (!cv && out_t && !gmax && c < ldt)
        for (int p = g; p < P; p += 16) out_t[((long)b * P + p) * ldt + c] = fpm::from_f<T>(0.f);
    if (gmax) {
        __syncthreads();
        red[g][cl] = mx;
        __syncthreads();
        if (g == 0 && cv) {
            float m = red[0][cl];
#pragma unroll
            for (int q = 1; q < 16; ++q) m = fmaxf(m, red[q][cl]);
            gmax[(long)b * Cn + c] = m;
        }
    }
}

// ks = sigmoid((final_row(gr) + final_col(gc)) / 2)   (ngm.py:406-412, mean_k = True)
__global__ __launch_bounds__(64) void afau_head_kernel(const float* __restrict__ gr, const float* __restrict__ gc,
                                                       int E, const float* __restrict__ r0w, const float* __restrict__ r0b,
                                                       const float* __restrict__ r2w, const float* __restrict__ r2b,
                                                       const float* __restrict__ c0w, const float* __restrict__ c0b,
                                                       const float* __restrict__ c2w, const float* __restrict__ c2b,
                                                       float* __restrict__ ks) {
    const int b = blockIdx.x, lane = threadIdx.x;
    float kr = 0.f, kc = 0.f;
    for (int m = 0; m < 8; ++m) {
        float sr = 0.f, sc = 0.f;
        for (int k = lane; k < E; k += 64) {
            sr += r0w[m * E + k] * gr[(long)b * E + k];
            sc += c0w[m * E + k] * gc[(long)b * E + k];
        }
        sr = fpm::warp_sum(sr) + r0b[m];
        sc = fpm::warp_sum(sc) + c0b[m];
        kr += r2w[m] * fmaxf(sr, 0.f);
        kc += c2w[m] * fmaxf(sc, 0.f);
    }
    kr += r2b[0];
    kc += c2b[0];
    if (lane == 0) ks[b] = 1.f / (1.f + expf(-((kr + kc) / 2.f)));
}

}  // namespace

extern "C" int fpm_crossset_attn_fwd(int dtype, const float* cost, long c_sb, long c_ld, int B, int n1max, int n2max,
                                     const int* n2, const float* Wv, int emb, const float* mix1w, const float* mix1b,
                                     const float* mix2w, const float* mix2b, void* out, void* stream) {
    FPM_CHECK_ARG(n2max <= emb, "crossset_attn: n2max > embedding dim");
    if (B == 0) return 0;
    dim3 grid(B, (n1max + 15) / 16);
    size_t sh = (size_t)(n2max * 20 + 16 * n2max) * 4;
    FPM_CHECK_ARG(sh <= 160 * 1024, "crossset_attn: n2max %d needs %zu B of LDS", n2max, sh);
    hipStream_t st = (hipStream_t)stream;
    FPM_CHECK_ARG(n2max <= 640, "crossset_attn: n2max %d > 640", n2max);
#define FPM_ATT(TT, NJ)                                                                                      \
    do {                                                                                                     \
        if (sh > 64 * 1024)                                                                                  \
            (void)hipFuncSetAttribute((const void*)afau_row_attn_kernel<TT, NJ>,                             \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);                   \
        hipLaunchKernelGGL((afau_row_attn_kernel<TT, NJ>), grid, dim3(256), sh, st, cost, c_sb, c_ld, n1max, n2max, \
                           n2, Wv, emb, mix1w, mix1b, mix2w, mix2b, (TT*)out);                               \
    } while (0)
    if (dtype == 0) { if (n2max <= 256) FPM_ATT(float, 4); else FPM_ATT(float, 10); }
    else { if (n2max <= 256) FPM_ATT(bf16_t, 4); else FPM_ATT(bf16_t, 10); }
#undef FPM_ATT
    return fpm::check_launch("fpm_crossset_attn_fwd");
}

extern "C" int fpm_instnorm(int dtype, const float* in1, const float* in2, int B, int P, int Cn, const int* nvalid,
                            const float* onehot_bias, const float* w, const float* bias, float eps, float* out_f,
                            void* out_t, int ldt, float* gmax, void* stream) {
    if (B == 0) return 0;
    if (ldt <= 0) ldt = Cn;
    FPM_CHECK_ARG(ldt >= Cn, "instnorm: ldt %d < Cn %d", ldt, Cn);
    const int cols = ldt > Cn ? ldt : Cn;
    dim3 grid(B, (cols + 63) / 64);
    FPM_CHECK_ARG(P <= 640, "instnorm: P=%d > 640 positions", P);
    hipStream_t st = (hipStream_t)stream;
#define FPM_IN(TT, NV)                                                                                     \
    hipLaunchKernelGGL((instnorm_kernel<TT, NV>), grid, dim3(1024), 0, st, in1, in2, P, Cn, nvalid, onehot_bias, w, \
                       bias, eps, out_f, (TT*)out_t, ldt, gmax)
    if (dtype == 0) { if (P <= 256) FPM_IN(float, 16); else FPM_IN(float, 40); }
    else { if (P <= 256) FPM_IN(bf16_t, 16); else FPM_IN(bf16_t, 40); }
#undef FPM_IN
    return fpm::check_launch("fpm_instnorm");
}

extern "C" int fpm_afau_head(const float* gr, const float* gc, int B, int E, const float* r0w, const float* r0b,
                             const float* r2w, const float* r2b, const float* c0w, const float* c0b, const float* c2w,
                             const float* c2b, float* ks, void* stream) {
    if (B == 0) return 0;
    hipLaunchKernelGGL(afau_head_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, gr, gc, E, r0w, r0b, r2w, r2b, c0w,
                       c0b, c2w, c2b, ks);
    return fpm::check_launch("fpm_afau_head");
}
