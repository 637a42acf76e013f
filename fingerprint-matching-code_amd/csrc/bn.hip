// Training-mode BatchNorm2d fused with the ReLU in front of it, for the MatchClassifier's
// conv -> ReLU -> BatchNorm2d -> MaxPool blocks (reference src/model/ngm.py:90-99; torch
// F.batch_norm(training=True) semantics: batch statistics with the biased variance for the
// normalisation, running_var updated with the unbiased one, momentum update of the running
// buffers).  Replaces MIOpen's BatchNorm fwd/bwd-train kernels in the training step
// (profiles/r02_train_kernel_stats: 9 % of the step on B = 64 x 16 x 256 x 256 maps).
//
// NCHW fp32.  Per-channel sums are deterministic: one workgroup per (sample, channel) plane sums
// it (float4 loads, wave shuffle trees, fixed order) into part[n][c][2]; a second pass combines the N
// partials per channel in order in fp64.  Forward statistics are centred: each plane stores its sum
// and the sum of squares about its own mean (a second pass over the plane), and the channel pass
// merges them with Chan's formula, M2 = sum_n [M2_n + HW (mean_n - mean)^2] -- no E[r^2] - mean^2
// cancellation when |mean| >> std (torch's batch_norm is Welford-based).
//   forward:  r = relu(x);  mean, var over (n, h, w);  y = (r - mean) * invstd * gamma + beta
//   backward: xhat = (r - mean) * invstd;  sdy = sum dy, sdx = sum dy * xhat (per channel);
//             dx = [x > 0] * gamma * invstd * (dy - sdy / M - xhat * sdx / M);
//             dgamma = sdx, dbeta = sdy
#include "fpm_common.h"

namespace {

constexpr int BN_T = 256;

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// MODE 0: sums of relu(x), relu(x)^2;  MODE 1: sums of dy, dy * xhat(x)
template <int MODE>
__global__ __launch_bounds__(BN_T) void bn_plane_sums_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                             int C, long HW, const float* __restrict__ stats,
                                                             float* __restrict__ part) {
    __shared__ float red[2][BN_T / 64];
    const int nc = blockIdx.x, c = nc % C;
    const float* xp = x + (long)nc * HW;
    const float* dp = MODE == 1 ? dy + (long)nc * HW : nullptr;
    float mean = 0.f, inv = 0.f;
    if (MODE == 1) {
        mean = stats[2 * c];
        inv = stats[2 * c + 1];
    }
    // pass 0 (MODE 0): plane sum; MODE 0 pass 1: squares about the plane mean; MODE 1: both sums
    float a0 = 0.f, a1 = 0.f;
    float pm = 0.f;
    auto acc = [&](int pass, float xv, float dv) {
        const float r = fmaxf(xv, 0.f);
        if (MODE == 0) {
            if (pass == 0) {
                a0 += r;
            } else {
                const float d = r - pm;
                a1 = fmaf(d, d, a1);
            }
        } else {
            a0 += dv;
            a1 = fmaf(dv, (r - mean) * inv, a1);
        }
    };
    auto sweep = [&](int pass) {
        if ((HW & 3) == 0) {
            for (long i = 4 * (long)threadIdx.x; i < HW; i += 4 * BN_T) {
                const float4 v = *(const float4*)(xp + i);
                float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
                if (MODE == 1) d = *(const float4*)(dp + i);
                acc(pass, v.x, d.x); acc(pass, v.y, d.y); acc(pass, v.z, d.z); acc(pass, v.w, d.w);
            }
        } else {
            for (long i = threadIdx.x; i < HW; i += BN_T) acc(pass, xp[i], MODE == 1 ? dp[i] : 0.f);
        }
    };
    // fixed-order block sum of v (every thread gets the result)
    auto bsum = [&](float v, int slot) {
        v = wsum(v);
        if ((threadIdx.x & 63) == 0) red[slot][threadIdx.x >> 6] = v;
        __syncthreads();
        float s = 0.f;
        for (int k = 0; k < BN_T / 64; ++k) s += red[slot][k];
        return s;
    };
    sweep(0);
    const float s0 = bsum(a0, 0);
    if (MODE == 0) {
        pm = s0 / (float)HW;
        sweep(1);
    }
    const float s1 = bsum(a1, 1);
    if (threadIdx.x == 0) {
        part[2 * (long)nc] = s0;
        part[2 * (long)nc + 1] = s1;
    }
}

// per channel (one thread each): combine the N plane partials in order (fp64).
// MODE 0 -> stats = (mean, invstd), running buffers updated; MODE 1 -> dgamma, dbeta, and
// coef = (gamma * invstd, sdy / M, sdx / M) for the dx pass
template <int MODE>
__global__ void bn_channel_kernel(const float* __restrict__ part, int N, int C, long HW, float eps, float momentum,
                                  float* __restrict__ stats, float* running_mean, float* running_var,
                                  const float* __restrict__ gamma, float* __restrict__ dgamma,
                                  float* __restrict__ dbeta, float* __restrict__ coef) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double s0 = 0.0, s1 = 0.0;
    for (int n = 0; n < N; ++n) {
        s0 += (double)part[2 * ((long)n * C + c)];
        s1 += (double)part[2 * ((long)n * C + c) + 1];
    }
    const double M = (double)N * (double)HW;
    if (MODE == 0) {
        const double mean = s0 / M;
        // Chan merge of the planes' centred sums (the plane means as the fp32 values pass 1 used)
        double m2 = 0.0;
        for (int n = 0; n < N; ++n) {
            const double d = (double)(part[2 * ((long)n * C + c)] / (float)HW) - mean;
            m2 += (double)part[2 * ((long)n * C + c) + 1] + (double)HW * d * d;
        }
        const double var = m2 / M;
        stats[2 * c] = (float)mean;
        stats[2 * c + 1] = (float)(1.0 / sqrt(var + (double)eps));
        if (running_mean) {
            const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
            running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
            running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
        }
    } else {
        dbeta[c] = (float)s0;
        dgamma[c] = (float)s1;
        coef[3 * c] = gamma[c] * stats[2 * c + 1];
        coef[3 * c + 1] = (float)(s0 / M);
        coef[3 * c + 2] = (float)(s1 / M);
    }
}

// grid (chunks of 4 * BN_T elements, N * C planes): the channel is uniform per workgroup
__global__ __launch_bounds__(BN_T) void bn_apply_kernel(const float* __restrict__ x, int C, long HW,
                                                        const float* __restrict__ stats,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float* __restrict__ y) {
    const long nc = blockIdx.y;
    const int c = (int)(nc % C);
    const float g = gamma[c] * stats[2 * c + 1], bb = beta[c] - stats[2 * c] * g;
    const float* xp = x + nc * HW;
    float* yp = y + nc * HW;
    const long i = ((long)blockIdx.x * BN_T + threadIdx.x) * 4;
    if ((HW & 3) == 0) {
        if (i >= HW) return;
        const float4 v = *(const float4*)(xp + i);
        *(float4*)(yp + i) = make_float4(fmaf(fmaxf(v.x, 0.f), g, bb), fmaf(fmaxf(v.y, 0.f), g, bb),
                                         fmaf(fmaxf(v.z, 0.f), g, bb), fmaf(fmaxf(v.w, 0.f), g, bb));
    } else {
        for (long k = i; k < i + 4 && k < HW; ++k) yp[k] = fmaf(fmaxf(xp[k], 0.f), g, bb);
    }
}

__global__ __launch_bounds__(BN_T) void bn_dx_kernel(const float* __restrict__ x, const float* __restrict__ dy, int C,
                                                     long HW, const float* __restrict__ stats,
                                                     const float* __restrict__ coef, float* __restrict__ dx) {
    const long nc = blockIdx.y;
    const int c = (int)(nc % C);
    const float mean = stats[2 * c], inv = stats[2 * c + 1];
    const float k0 = coef[3 * c], k1 = coef[3 * c + 1], k2 = coef[3 * c + 2];
    const float* xp = x + nc * HW;
    const float* dp = dy + nc * HW;
    float* op = dx + nc * HW;
    auto one = [&](float xv, float dv) {
        const float xhat = (fmaxf(xv, 0.f) - mean) * inv;
        const float g = k0 * (dv - k1 - xhat * k2);
        return xv > 0.f ? g : 0.f;
    };
    const long i = ((long)blockIdx.x * BN_T + threadIdx.x) * 4;
    if ((HW & 3) == 0) {
        if (i >= HW) return;
        const float4 v = *(const float4*)(xp + i), d = *(const float4*)(dp + i);
        *(float4*)(op + i) = make_float4(one(v.x, d.x), one(v.y, d.y), one(v.z, d.z), one(v.w, d.w));
    } else {
        for (long k = i; k < i + 4 && k < HW; ++k) op[k] = one(xp[k], dp[k]);
    }
}

}  // namespace

extern "C" long fpm_bn_ws_floats(int N, int C) { return 2L * N * C + 5L * C; }

// x: conv output (N, C, HW); y = BN(relu(x)); stats (2C): (mean, invstd) kept for the backward.
// running_mean / running_var (nullable) get the momentum update.  ws: fpm_bn_ws_floats floats.
extern "C" int fpm_bn_relu_train_fwd(const float* x, int N, int C, long HW, const float* gamma, const float* beta,
                                     float eps, float momentum, float* running_mean, float* running_var, float* y,
                                     float* stats, float* ws, void* stream) {
    FPM_CHECK_ARG(N > 0 && C > 0 && HW > 0, "bn_relu_train_fwd: bad sizes");
    hipStream_t st = (hipStream_t)stream;
    float* part = ws;
    hipLaunchKernelGGL(bn_plane_sums_kernel<0>, dim3((unsigned)(N * C)), dim3(BN_T), 0, st, x, nullptr, C, HW, nullptr,
                       part);
    hipLaunchKernelGGL(bn_channel_kernel<0>, dim3((C + 63) / 64), dim3(64), 0, st, part, N, C, HW, eps, momentum, stats,
                       running_mean, running_var, nullptr, nullptr, nullptr, nullptr);
    const dim3 grid((unsigned)((HW + 4 * BN_T - 1) / (4 * BN_T)), (unsigned)(N * C));
    hipLaunchKernelGGL(bn_apply_kernel, grid, dim3(BN_T), 0, st, x, C, HW, stats, gamma, beta, y);
    return fpm::check_launch("fpm_bn_relu_train_fwd");
}

// dy: gradient of y; dx: gradient of x (the conv output, through the ReLU); dgamma, dbeta (C).
extern "C" int fpm_bn_relu_train_bwd(const float* x, const float* dy, int N, int C, long HW, const float* gamma,
                                     const float* stats, float* dx, float* dgamma, float* dbeta, float* ws,
                                     void* stream) {
    FPM_CHECK_ARG(N > 0 && C > 0 && HW > 0, "bn_relu_train_bwd: bad sizes");
    hipStream_t st = (hipStream_t)stream;
    float* part = ws;
    float* coef = ws + 2L * N * C;
    hipLaunchKernelGGL(bn_plane_sums_kernel<1>, dim3((unsigned)(N * C)), dim3(BN_T), 0, st, x, dy, C, HW, stats, part);
    hipLaunchKernelGGL(bn_channel_kernel<1>, dim3((C + 63) / 64), dim3(64), 0, st, part, N, C, HW, 0.f, 0.f,
                       const_cast<float*>(stats), nullptr, nullptr, gamma, dgamma, dbeta, coef);
    const dim3 grid((unsigned)((HW + 4 * BN_T - 1) / (4 * BN_T)), (unsigned)(N * C));
    hipLaunchKernelGGL(bn_dx_kernel, grid, dim3(BN_T), 0, st, x, dy, C, HW, stats, coef, dx);
    return fpm::check_launch("fpm_bn_relu_train_bwd");
}
