// MatchClassifier (reference ngm.py:75-106) on matched_sim = s * perm_mat (ngm.py:451-455):
//   [conv3x3(1->16,pad 1) -> ReLU -> BN(eval) -> MaxPool2] -> [conv3x3(16->32) -> ReLU -> BN -> MaxPool2]
//   -> global average pool -> Linear(32->1) -> logit (sigmoid applied for cls_prob).
// fp32 throughout; stage 1 (direct conv) fuses the s*perm product, stage 2 runs conv2 as an
// implicit GEMM on the fp32 matrix cores and fuses the average pool into per-block partial sums
// (deterministic, reduced by the head kernel).
#include "fpm_common.h"

namespace {

// P1[b][c][ph][pw] fp32 (BF = false) or P1[b][ph][pw][c] bf16 (BF = true: the channel-minor
// operand layout of the bf16 conv2), H1 = H/2, W1 = W/2 (floor)
template <bool BF>
__global__ __launch_bounds__(256) void cls_stage1_kernel(const float* __restrict__ s, const float* __restrict__ perm,
                                                         int H, int W, const float* __restrict__ w1,
                                                         const float* __restrict__ b1, const float* __restrict__ bn_sc,
                                                         const float* __restrict__ bn_sh, void* __restrict__ P1v) {
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
    float outc[16];
#pragma unroll
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
        outc[ch] = mx;
    }
    if (BF) {
        uint32_t w[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) w[q] = (uint32_t)fpm::f2bf(outc[2 * q]) | ((uint32_t)fpm::f2bf(outc[2 * q + 1]) << 16);
        uint4* o = (uint4*)((bf16_t*)P1v + (((long)b * H1 + ph) * W1 + pw) * 16);
        o[0] = make_uint4(w[0], w[1], w[2], w[3]);
        o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
        float* P1 = (float*)P1v;
#pragma unroll
        for (int ch = 0; ch < 16; ++ch) P1[(((long)b * 16 + ch) * H1 + ph) * W1 + pw] = outc[ch];
    }
}

// conv2 (16 -> 32, 3x3, pad 1) + ReLU + BN + MaxPool2 + partial sums of the pooled map per channel,
// as an implicit GEMM on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32 products):
// out^T[oc][pos] = W2[oc][k] . im2col[k][pos], k = ci*9 + ky*3 + kx (144 = 36 K-steps of 4).
// Block = one pair, a 16 x 32 tile of pre-pool positions (8 x 16 pooled pixels); the 16-channel
// input tile with its 1-pixel halo is staged in LDS.  Wave w owns pre-pool rows 4w..4w+3: two
// row pairs x two 16-column halves; each lane holds the B operand (one im2col entry) per K-step.
constexpr int C2_TY = 16, C2_TX = 32, C2_LY = C2_TY + 2, C2_LX = C2_TX + 2;
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void cls_stage2_kernel(const float* __restrict__ P1, int H1, int W1,
                                                         const float* __restrict__ w2, const float* __restrict__ b2,
                                                         const float* __restrict__ bn_sc, const float* __restrict__ bn_sh,
                                                         float* __restrict__ part) {
    __shared__ float tin[16 * C2_LY * C2_LX];
    __shared__ float red[4][32];
    const int H2 = H1 / 2, W2 = W1 / 2;
    const int tiles_x = (2 * W2 + C2_TX - 1) / C2_TX;
    const int b = blockIdx.y;
    const int ty = blockIdx.x / tiles_x, tx = blockIdx.x - ty * tiles_x;
    const int y0 = ty * C2_TY, x0 = tx * C2_TX;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, col = lane & 15;
    const float* src = P1 + (long)b * 16 * H1 * W1;
    for (int k = tid; k < 16 * C2_LY * C2_LX; k += 256) {
        const int ci = k / (C2_LY * C2_LX), rem = k - ci * (C2_LY * C2_LX);
        const int yy = rem / C2_LX, xx = rem - yy * C2_LX;
        const int y = y0 - 1 + yy, x = x0 - 1 + xx;
        tin[k] = (y >= 0 && y < H1 && x >= 0 && x < W1) ? src[((long)ci * H1 + y) * W1 + x] : 0.f;
    }
    // A operands: W2[16 mt + col][4 s + g]
    float wa[2][36];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int s = 0; s < 36; ++s) wa[mt][s] = w2[(16 * mt + col) * 144 + 4 * s + g];
    float bsh[2][4], bsc[2][4], bsf[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int oc = 16 * mt + 4 * g + r;
            bsh[mt][r] = b2[oc];
            bsc[mt][r] = bn_sc[oc];
            bsf[mt][r] = bn_sh[oc];
        }
    __syncthreads();
    float sums[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int rp = 0; rp < 2; ++rp) {
        const int r0 = wave * 4 + rp * 2;                 // tile row of the pair's first row
#pragma unroll
        for (int xh = 0; xh < 2; ++xh) {
            f32x4_t acc[2][2];                            // [mt][row of the pair]
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 2; ++q) acc[mt][q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            const int xl = xh * 16 + col;                 // tile column of this lane's position
#pragma unroll
            for (int s = 0; s < 36; ++s) {
                const int k = 4 * s + g, ci = k / 9, t = k - ci * 9, ky = t / 3, kx = t - ky * 3;
                const float* base = tin + (ci * C2_LY + r0 + ky) * C2_LX + xl + kx;
                const float v0 = base[0], v1 = base[C2_LX];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[mt][s], v0, acc[mt][0], 0, 0, 0);
                    acc[mt][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[mt][s], v1, acc[mt][1], 0, 0, 0);
                }
            }
            // ReLU -> BN -> 2x2 max (rows in acc[.][0/1], columns in lanes col, col ^ 1)
            const int py = (y0 + r0) / 2, px = (x0 + xl) / 2;
            const bool ok = ((col & 1) == 0) && py < H2 && px < W2;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float a = fmaxf(acc[mt][0][r] + bsh[mt][r], 0.f) * bsc[mt][r] + bsf[mt][r];
                    float c = fmaxf(acc[mt][1][r] + bsh[mt][r], 0.f) * bsc[mt][r] + bsf[mt][r];
                    float m = fmaxf(a, c);
                    m = fmaxf(m, __shfl_xor(m, 1));
                    if (ok) sums[mt][r] += m;
                }
        }
    }
    // per-channel block sums: over the 16 columns of each row group, then the 4 waves
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = sums[mt][r];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (col == 0) red[wave][16 * mt + 4 * g + r] = v;
        }
    __syncthreads();
    if (tid < 32)
        part[((long)b * gridDim.x + blockIdx.x) * 32 + tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}

// bf16 mode: the same implicit GEMM on v_mfma_f32_16x16x16_bf16 with K ordered tap-major,
// channel-minor (k = tap * 16 + ci): one K-step = one 3x3 tap over all 16 input channels, so a
// lane's B operand (4 channels of one pixel) is one 8-byte LDS read from the channel-minor bf16
// tile, and the 144-long K is 9 MFMAs per output fragment instead of 36.
typedef short bf16x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void cls_stage2_bf16_kernel(const bf16_t* __restrict__ P1, int H1, int W1,
                                                              const float* __restrict__ w2, const float* __restrict__ b2,
                                                              const float* __restrict__ bn_sc,
                                                              const float* __restrict__ bn_sh, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) bf16_t tin[C2_LY * C2_LX * 16];
    __shared__ float red[4][32];
    const int H2 = H1 / 2, W2 = W1 / 2;
    const int tiles_x = (2 * W2 + C2_TX - 1) / C2_TX;
    const int b = blockIdx.y;
    const int ty = blockIdx.x / tiles_x, tx = blockIdx.x - ty * tiles_x;
    const int y0 = ty * C2_TY, x0 = tx * C2_TX;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, col = lane & 15;
    const bf16_t* src = P1 + (long)b * H1 * W1 * 16;
    // halo tile, 32 B per pixel (16 channels), two 16-B pieces per pixel
    for (int k = tid; k < C2_LY * C2_LX * 2; k += 256) {
        const int px = k >> 1, h = k & 1;
        const int yy = px / C2_LX, xx = px - yy * C2_LX;
        const int y = y0 - 1 + yy, x = x0 - 1 + xx;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (y >= 0 && y < H1 && x >= 0 && x < W1) v = *(const uint4*)(src + ((long)y * W1 + x) * 16 + 8 * h);
        *(uint4*)(tin + px * 16 + 8 * h) = v;
    }
    // A operands: W2[16 mt + col][ci = 4g .. 4g+3][tap t] as 4 bf16
    bf16x4_t wa[2][9];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            bf16x4_t a;
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = (short)fpm::f2bf(w2[(16 * mt + col) * 144 + (4 * g + j) * 9 + t]);
            wa[mt][t] = a;
        }
    float bsh[2][4], bsc[2][4], bsf[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int oc = 16 * mt + 4 * g + r;
            bsh[mt][r] = b2[oc];
            bsc[mt][r] = bn_sc[oc];
            bsf[mt][r] = bn_sh[oc];
        }
    __syncthreads();
    float sums[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int rp = 0; rp < 2; ++rp) {
        const int r0 = wave * 4 + rp * 2;
#pragma unroll
        for (int xh = 0; xh < 2; ++xh) {
            f32x4_t acc[2][2];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 2; ++q) acc[mt][q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            const int xl = xh * 16 + col;
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int ky = t / 3, kx = t - ky * 3;
                const bf16_t* base = tin + ((r0 + ky) * C2_LX + xl + kx) * 16 + 4 * g;
                const bf16x4_t v0 = *(const bf16x4_t*)base;
                const bf16x4_t v1 = *(const bf16x4_t*)(base + C2_LX * 16);
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wa[mt][t], v0, acc[mt][0], 0, 0, 0);
                    acc[mt][1] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wa[mt][t], v1, acc[mt][1], 0, 0, 0);
                }
            }
            const int py = (y0 + r0) / 2, px = (x0 + xl) / 2;
            const bool ok = ((col & 1) == 0) && py < H2 && px < W2;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float a = fmaxf(acc[mt][0][r] + bsh[mt][r], 0.f) * bsc[mt][r] + bsf[mt][r];
                    float c = fmaxf(acc[mt][1][r] + bsh[mt][r], 0.f) * bsc[mt][r] + bsf[mt][r];
                    float m = fmaxf(a, c);
                    m = fmaxf(m, __shfl_xor(m, 1));
                    if (ok) sums[mt][r] += m;
                }
        }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = sums[mt][r];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (col == 0) red[wave][16 * mt + 4 * g + r] = v;
        }
    __syncthreads();
    if (tid < 32)
        part[((long)b * gridDim.x + blockIdx.x) * 32 + tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
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

static long cls2_blocks(int H1, int W1) {
    const long H2 = H1 / 2, W2 = W1 / 2;
    return ((2 * H2 + C2_TY - 1) / C2_TY) * ((2 * W2 + C2_TX - 1) / C2_TX);
}

extern "C" long fpm_match_cls_ws_floats(int B, int H, int W) {
    long H1 = H / 2, W1 = W / 2;
    return (long)B * 16 * H1 * W1 + (long)B * cls2_blocks((int)H1, (int)W1) * 32;
}

// bn*_sc = gamma / sqrt(running_var + eps), bn*_sh = beta - running_mean * bn*_sc (host-folded)
// dtype 0: fp32 conv2 (exact fp32 products), 1: bf16 conv2 operands (fp32 accumulation)
extern "C" int fpm_match_cls_fwd(int dtype, const float* s, const float* perm, int B, int H, int W, const float* w1,
                                 const float* b1, const float* bn1_sc, const float* bn1_sh, const float* w2,
                                 const float* b2, const float* bn2_sc, const float* bn2_sh, const float* fcw,
                                 const float* fcb, float* ws, float* logits, float* prob, void* stream) {
    FPM_CHECK_ARG(H >= 4 && W >= 4, "match_cls: H, W must be >= 4");
    FPM_CHECK_ARG(dtype == 0 || dtype == 1, "match_cls: bad dtype");
    if (B == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int H1 = H / 2, W1 = W / 2, H2 = H1 / 2, W2 = W1 / 2;
    float* P1 = ws;
    const long nblk = cls2_blocks(H1, W1);
    float* part = ws + (long)B * 16 * H1 * W1;
    const dim3 g1((unsigned)(((long)H1 * W1 + 255) / 256), B);
    if (dtype == 1) {
        hipLaunchKernelGGL(cls_stage1_kernel<true>, g1, dim3(256), 0, st, s, perm, H, W, w1, b1, bn1_sc, bn1_sh,
                           (void*)P1);
        hipLaunchKernelGGL(cls_stage2_bf16_kernel, dim3((unsigned)nblk, B), dim3(256), 0, st, (const bf16_t*)P1, H1, W1,
                           w2, b2, bn2_sc, bn2_sh, part);
    } else {
        hipLaunchKernelGGL(cls_stage1_kernel<false>, g1, dim3(256), 0, st, s, perm, H, W, w1, b1, bn1_sc, bn1_sh,
                           (void*)P1);
        hipLaunchKernelGGL(cls_stage2_kernel, dim3((unsigned)nblk, B), dim3(256), 0, st, P1, H1, W1, w2, b2, bn2_sc,
                           bn2_sh, part);
    }
    hipLaunchKernelGGL(cls_head_kernel, dim3(B), dim3(64), 0, st, part, (int)nblk, (long)H2 * W2, fcw, fcb, logits,
                       prob);
    return fpm::check_launch("fpm_match_cls_fwd");
}
