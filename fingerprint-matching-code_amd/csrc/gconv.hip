// Gconv (src/model/gcn.py:8-38): x' = norm1(A) . relu(a_fc x) + relu(u_fc x), batched (b, n, n) x
// (b, n, d).  Not used by Net; a thin fp32 kernel set for API completeness.
//   1. both linears in one pass: H[r][0:dout] = relu(x_r Wa^T + ba), H[r][dout:2dout] = relu(x_r Wu^T + bu)
//   2. column L1 norms of A (F.normalize(A, p=1, dim=-2): divide by max(sum_i |A_ij|, 1e-12))
//   3. out[b,i,o] = sum_j (A[b,i,j] / den[b,j]) * H[b,j,o] + H[b,i,dout+o]
#include "fpm_common.h"

namespace {

__global__ void gconv_linear_kernel(const float* __restrict__ x, long rows, int din, int dout2,
                                    const float* __restrict__ w, const float* __restrict__ bias,
                                    float* __restrict__ H) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * dout2) return;
    const long r = t / dout2;
    const int o = (int)(t - r * dout2);
    const float* xr = x + r * din;
    const float* wo = w + (long)o * din;
    float s = 0.f;
    for (int k = 0; k < din; ++k) s = fmaf(xr[k], wo[k], s);
    H[t] = fmaxf(s + bias[o], 0.f);
}

__global__ void gconv_colnorm_kernel(const float* __restrict__ A, int B, int n, int norm, float* __restrict__ den) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B * n) return;
    const long b = t / n, j = t - b * n;
    if (!norm) {
        den[t] = 1.f;
        return;
    }
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += fabsf(A[(b * n + i) * n + j]);
    den[t] = fmaxf(s, 1e-12f);
}

__global__ void gconv_agg_kernel(const float* __restrict__ A, const float* __restrict__ den,
                                 const float* __restrict__ H, int B, int n, int dout, int norm,
                                 float* __restrict__ out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B * n * dout) return;
    const int o = (int)(t % dout);
    const long bi = t / dout;
    const long b = bi / n;
    const float* arow = A + bi * n;
    const float* Hb = H + b * n * 2 * dout;
    float s = 0.f;
    for (int j = 0; j < n; ++j) {
        const float a = norm ? arow[j] / den[b * n + j] : arow[j];
        s = fmaf(a, Hb[(long)j * 2 * dout + o], s);
    }
    out[t] = s + H[bi * 2 * dout + dout + o];
}

}  // namespace

extern "C" long fpm_gconv_ws_floats(int B, int n, int dout) { return (long)B * n * (2L * dout + 1); }

// W: (2*dout, din) = [a_fc.weight; u_fc.weight], bias (2*dout) = [a_fc.bias; u_fc.bias]
extern "C" int fpm_gconv_fwd(const float* A, const float* x, int B, int n, int din, int dout, const float* W,
                             const float* bias, int norm, float* ws, float* out, void* stream) {
    FPM_CHECK_ARG(B >= 0 && n >= 0 && din > 0 && dout > 0, "gconv: bad sizes");
    if (B == 0 || n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    float* H = ws;
    float* den = ws + (long)B * n * 2 * dout;
    const long rows = (long)B * n;
    hipLaunchKernelGGL(gconv_linear_kernel, dim3((unsigned)((rows * 2 * dout + 255) / 256)), dim3(256), 0, st, x,
                       rows, din, 2 * dout, W, bias, H);
    hipLaunchKernelGGL(gconv_colnorm_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, A, B, n, norm,
                       den);
    hipLaunchKernelGGL(gconv_agg_kernel, dim3((unsigned)((rows * dout + 255) / 256)), dim3(256), 0, st, A, den, H, B,
                       n, dout, norm, out);
    return fpm::check_launch("fpm_gconv_fwd");
}
