// MatchClassifier (reference ngm.py:75-106) on matched_sim = s * perm_mat (ngm.py:451-455):
//   [conv3x3(1->16,pad 1) -> ReLU -> BN(eval) -> MaxPool2] -> [conv3x3(16->32) -> ReLU -> BN -> MaxPool2]
//   -> global average pool -> Linear(32->1) -> logit (sigmoid applied for cls_prob).
// Direct convolutions in fp32; stage 1 fuses the s*perm product, stage 2 fuses the average pool
// into per-block partial sums (deterministic, reduced by the head kernel).
#include "fpm_common.h"

namespace {

// P1[b][c][ph][pw], H1 = H/2, W1 = W/2 (floor)
__global__ __launch_bounds__(256) void cls_stage1_kernel(const float* __restrict__ s, const float* __restrict__ perm,
                                                         int H, int W, const float* __restrict__ w1,
                                                         const float* __restrict__ b1, const float* __restrict__ bn_sc,
                                                         const float* __restrict__ bn_sh, float* __restrict__ P1) {
    __shared__ float wsh[16 * 9 + 16 * 3];
    for (int k = threadIdx.x; k < 16 * 9; k += 256) wsh[k] = w1[k];
    for (int k = threadIdx.x; k < 16; k += 256) {
        wsh[144 + k] = b1[k];
        wsh[160 + k] = bn_sc[k];
        wsh[176 + k] = bn_sh[k];
    }
    __syncthreads();
    const int H1 = H / 2, W1 = W / 2;
    const int b = blockIdx.y;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long)H1 * W1) return;
    const int ph = (int)(idx / W1), pw = (int)(idx - (long)ph * W1);
    const float* S = s + (long)b * H * W;
    const float* Pm = perm + (long)b * H * W;
    float in[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            int y = 2 * ph - 1 + r, x = 2 * pw - 1 + c;
            in[r][c] = (y >= 0 && y < H && x >= 0 && x < W) ? S[(long)y * W + x] * Pm[(long)y * W + x] : 0.f;
        }
    for (int ch = 0; ch < 16; ++ch) {
        float mx = -INFINITY;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                float acc = 0.f;
#pragma unroll
                for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx) acc += wsh[ch * 9 + ky * 3 + kx] * in[dy + ky][dx + kx];
                acc += wsh[144 + ch];
                acc = fmaxf(acc, 0.f);
                acc = acc * wsh[160 + ch] + wsh[176 + ch];
                mx = fmaxf(mx, acc);
            }
        P1[(((long)b * 16 + ch) * H1 + ph) * W1 + pw] = mx;
    }
}

// conv2 + ReLU + BN + MaxPool2, then partial sums of the pooled map per channel.
// thread = (pooled pixel, channel group of 8); block sums written to part[b][blk][32]
__global__ __launch_bounds__(256) void cls_stage2_kernel(const float* __restrict__ P1, int H1, int W1,
                                                         const float* __restrict__ w2, const float* __restrict__ b2,
                                                         const float* __restrict__ bn_sc, const float* __restrict__ bn_sh,
                                                         float* __restrict__ part) {
    __shared__ float wsh[32 * 16 * 9];
    __shared__ float red[256][8];
    for (int k = threadIdx.x; k < 32 * 144; k += 256) wsh[k] = w2[k];
    __syncthreads();
    const int H2 = H1 / 2, W2 = W1 / 2;
    const int b = blockIdx.y;
    const int cg = threadIdx.x & 3;         // channels 8*cg .. 8*cg+7
    const long pix = (long)blockIdx.x * 64 + (threadIdx.x >> 2);
    float sums[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) sums[k] = 0.f;
    if (pix < (long)H2 * W2) {
        const int ph = (int)(pix / W2), pw = (int)(pix - (long)ph * W2);
        float acc[8][4];
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[k][q] = 0.f;
        for (int ci = 0; ci < 16; ++ci) {
            float in[4][4];
            const float* src = P1 + ((long)b * 16 + ci) * H1 * W1;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    int y = 2 * ph - 1 + r, x = 2 * pw - 1 + c;
                    in[r][c] = (y >= 0 && y < H1 && x >= 0 && x < W1) ? src[(long)y * W1 + x] : 0.f;
                }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float* wk = wsh + ((cg * 8 + k) * 16 + ci) * 9;
#pragma unroll
                for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 2; ++dx) {
                        float a = acc[k][dy * 2 + dx];
#pragma unroll
                        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                            for (int kx = 0; kx < 3; ++kx) a += wk[ky * 3 + kx] * in[dy + ky][dx + kx];
                        acc[k][dy * 2 + dx] = a;
                    }
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int ch = cg * 8 + k;
            float mx = -INFINITY;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float v = fmaxf(acc[k][q] + b2[ch], 0.f);
                v = v * bn_sc[ch] + bn_sh[ch];
                mx = fmaxf(mx, v);
            }
            sums[k] = mx;
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[threadIdx.x][k] = sums[k];
    __syncthreads();
    if (threadIdx.x < 32) {
        const int ch = threadIdx.x, g = ch >> 3, k = ch & 7;
        float s = 0.f;
        for (int t = g; t < 256; t += 4) s += red[t][k];
        part[((long)b * gridDim.x + blockIdx.x) * 32 + ch] = s;
    }
}

__global__ __launch_bounds__(64) void cls_head_kernel(const float* __restrict__ part, int nblk, long npix,
                                                      const float* __restrict__ fcw, const float* __restrict__ fcb,
                                                      float* __restrict__ logits, float* __restrict__ prob) {
    const int b = blockIdx.x, lane = threadIdx.x;
    float v = 0.f;
    if (lane < 32) {
        float s = 0.f;
        for (int k = 0; k < nblk; ++k) s += part[((long)b * nblk + k) * 32 + lane];
        v = (s / (float)npix) * fcw[lane];
    }
    v = fpm::warp_sum(v);
    if (lane == 0) {
        float l = v + fcb[0];
        logits[b] = l;
        if (prob) prob[b] = 1.f / (1.f + expf(-l));
    }
}

}  // namespace

extern "C" long fpm_match_cls_ws_floats(int B, int H, int W) {
    long H1 = H / 2, W1 = W / 2, H2 = H1 / 2, W2 = W1 / 2;
    long nblk = (H2 * W2 + 63) / 64;
    return (long)B * 16 * H1 * W1 + (long)B * nblk * 32;
}

// bn*_sc = gamma / sqrt(running_var + eps), bn*_sh = beta - running_mean * bn*_sc (host-folded)
extern "C" int fpm_match_cls_fwd(const float* s, const float* perm, int B, int H, int W, const float* w1, const float* b1,
                                 const float* bn1_sc, const float* bn1_sh, const float* w2, const float* b2,
                                 const float* bn2_sc, const float* bn2_sh, const float* fcw, const float* fcb, float* ws,
                                 float* logits, float* prob, void* stream) {
    FPM_CHECK_ARG(H >= 4 && W >= 4, "match_cls: H, W must be >= 4");
    if (B == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int H1 = H / 2, W1 = W / 2, H2 = H1 / 2, W2 = W1 / 2;
    float* P1 = ws;
    const long nblk = ((long)H2 * W2 + 63) / 64;
    float* part = ws + (long)B * 16 * H1 * W1;
    hipLaunchKernelGGL(cls_stage1_kernel, dim3((unsigned)(((long)H1 * W1 + 255) / 256), B), dim3(256), 0, st, s, perm,
                       H, W, w1, b1, bn1_sc, bn1_sh, P1);
    hipLaunchKernelGGL(cls_stage2_kernel, dim3((unsigned)nblk, B), dim3(256), 0, st, P1, H1, W1, w2, b2, bn2_sc, bn2_sh,
                       part);
    hipLaunchKernelGGL(cls_head_kernel, dim3(B), dim3(64), 0, st, part, (int)nblk, (long)H2 * W2, fcw, fcb, logits,
                       prob);
    return fpm::check_launch("fpm_match_cls_fwd");
}
