// Image front end of Net.forward after the CNN, src/model/ngm.py:235-248:
//   global  w = AdaptiveMaxPool2d(1)(edges)                               (ngm.py:238)
//   nodes/edges /= torch.norm(., dim=1)   (normalize_over_channels, ngm.py:65-67,241-243)
//   U = feature_align(nodes, P, ns, (320, 240)), F = feature_align(edges, ...)  (ngm.py:246-247)
//   x = [U || F] per keypoint                                             (concat_features, :70-72)
// feature_align / interp_2d / bilinear_interpolate: utils/feature_align.py:5-126, restated with
// its quirks: feat_size = feature.shape[1:3] = (H, W) is divided against ori_size = (320, 240) =
// (W, H), so x is scaled by H/320 but indexes the W axis (feature_align.py:57-62); corner indices
// are clamped before the gather, and a clamped-equal pair is pushed apart only for the weights
// (nearest-neighbour at the border, :100-110).  The interpolation is evaluated in fp32 with the
// reference's operation order and no FMA contraction: out = ((Ia*wa + Ib*wb) + Ic*wc) + Id*wd.
// Feature maps are read through (batch, channel, row, col) strides, so NCHW and channels_last
// (contiguous 1-KB pixel vectors, the layout the wave reads coalesced) both work.
//
// Kernels: pixel_norm (one wave per pixel, sum of squares over channels) -> align (one wave per
// keypoint, lane-strided channels: 4 corners of both maps, divided by the corner norms, blended,
// written as one 768-float row of the matcher's node-feature layout, zero rows for padding) and
// global_maxpool (thread per (image, channel)).  All three are L2/HBM-bound gathers.
#include "fpm_common.h"

namespace {

struct Map {
    const float* p;
    long sb, sc, sh, sw;
    int C, H, W;
};

__global__ __launch_bounds__(256) void pixel_norm_kernel(Map m, int B, float* __restrict__ norm) {
    const long wv = ((long)blockIdx.x * blockDim.x + threadIdx.x) / FPM_WAVE;
    const int lane = threadIdx.x & (FPM_WAVE - 1);
    const long npix = (long)B * m.H * m.W;
    if (wv >= npix) return;
    const long b = wv / ((long)m.H * m.W);
    const int r = (int)(wv - b * m.H * m.W);
    const int y = r / m.W, x = r - y * m.W;
    const float* base = m.p + b * m.sb + (long)y * m.sh + (long)x * m.sw;
    float s = 0.f;
    for (int c = lane; c < m.C; c += FPM_WAVE) {
        const float v = base[(long)c * m.sc];
        s = fmaf(v, v, s);
    }
    s = fpm::warp_sum(s);
    if (lane == 0) norm[wv] = sqrtf(s);
}

struct Corner {
    long off[4];  // a (y0,x0), b (y1,x0), c (y0,x1), d (y1,x1) pixel offsets in the norm array
    float w[4];
};

// bilinear_interpolate (feature_align.py:71-126) for one point already in feature-map units
__device__ __forceinline__ Corner corners(float x, float y, int H, int W) {
    const float fx0 = floorf(x), fy0 = floorf(y);
    float x0 = fminf(fmaxf(fx0, 0.f), (float)(W - 1));
    float x1 = fminf(fmaxf(__fadd_rn(fx0, 1.f), 0.f), (float)(W - 1));
    float y0 = fminf(fmaxf(fy0, 0.f), (float)(H - 1));
    float y1 = fminf(fmaxf(__fadd_rn(fy0, 1.f), 0.f), (float)(H - 1));
    const int ix0 = (int)x0, ix1 = (int)x1, iy0 = (int)y0, iy1 = (int)y1;
    Corner c;
    c.off[0] = (long)iy0 * W + ix0;
    c.off[1] = (long)iy1 * W + ix0;
    c.off[2] = (long)iy0 * W + ix1;
    c.off[3] = (long)iy1 * W + ix1;
    if (ix0 == ix1) {
        if (ix0 == 0) x0 -= 1.f;
        else x1 += 1.f;
    }
    if (iy0 == iy1) {
        if (iy0 == 0) y0 -= 1.f;
        else y1 += 1.f;
    }
    c.w[0] = __fmul_rn(__fsub_rn(x1, x), __fsub_rn(y1, y));
    c.w[1] = __fmul_rn(__fsub_rn(x1, x), __fsub_rn(y, y0));
    c.w[2] = __fmul_rn(__fsub_rn(x, x0), __fsub_rn(y1, y));
    c.w[3] = __fmul_rn(__fsub_rn(x, x0), __fsub_rn(y, y0));
    return c;
}

// interp_2d's point transform (feature_align.py:57-62), fp32 in torch's order:
// p = (P - step/2) / ori_size * feat_size with step = ori_size / feat_size, feat_size = (H, W)
__device__ __forceinline__ void to_map(float px, float py, float ox, float oy, int H, int W, float& x, float& y) {
    const float fs0 = (float)H, fs1 = (float)W;
    const float st0 = __fdiv_rn(ox, fs0), st1 = __fdiv_rn(oy, fs1);
    x = __fmul_rn(__fdiv_rn(__fsub_rn(px, __fdiv_rn(st0, 2.f)), ox), fs0);
    y = __fmul_rn(__fdiv_rn(__fsub_rn(py, __fdiv_rn(st1, 2.f)), oy), fs1);
}

__device__ __forceinline__ void interp_map(const Map& m, const float* __restrict__ nrm, long b, float px, float py,
                                           float ox, float oy, int lane, float* __restrict__ out) {
    float x, y;
    to_map(px, py, ox, oy, m.H, m.W, x, y);
    const Corner c = corners(x, y, m.H, m.W);
    const float* nb = nrm + b * m.H * m.W;
    float nv[4];
    const float* pp[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        nv[q] = nb[c.off[q]];
        const long yy = c.off[q] / m.W, xx = c.off[q] - yy * m.W;
        pp[q] = m.p + b * m.sb + yy * m.sh + xx * m.sw;
    }
    for (int ch = lane; ch < m.C; ch += FPM_WAVE) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = __fdiv_rn(pp[q][(long)ch * m.sc], nv[q]);
        float o = __fmul_rn(v[0], c.w[0]);
        o = __fadd_rn(o, __fmul_rn(v[1], c.w[1]));
        o = __fadd_rn(o, __fmul_rn(v[2], c.w[2]));
        o = __fadd_rn(o, __fmul_rn(v[3], c.w[3]));
        out[ch] = o;
    }
}

__global__ __launch_bounds__(256) void feature_align_kernel(Map nodes, Map edges, const float* __restrict__ nn_,
                                                            const float* __restrict__ ne_, const float* __restrict__ P,
                                                            const int* __restrict__ nv, int B, int nmax, float ox,
                                                            float oy, float* __restrict__ X, long ldx) {
    const long wv = ((long)blockIdx.x * blockDim.x + threadIdx.x) / FPM_WAVE;
    const int lane = threadIdx.x & (FPM_WAVE - 1);
    if (wv >= (long)B * nmax) return;
    const long b = wv / nmax;
    const int i = (int)(wv - b * nmax);
    float* row = X + wv * ldx;
    if (i >= nv[b]) {
        for (int ch = lane; ch < nodes.C + edges.C; ch += FPM_WAVE) row[ch] = 0.f;
        return;
    }
    const float px = P[wv * 2], py = P[wv * 2 + 1];
    interp_map(nodes, nn_, b, px, py, ox, oy, lane, row);
    interp_map(edges, ne_, b, px, py, ox, oy, lane, row + nodes.C);
}

__global__ void global_maxpool_kernel(Map m, int B, float* __restrict__ w) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B * m.C) return;
    const long b = t / m.C;
    const int c = (int)(t - b * m.C);
    const float* base = m.p + b * m.sb + (long)c * m.sc;
    float v = -INFINITY;
    for (int y = 0; y < m.H; ++y)
        for (int x = 0; x < m.W; ++x) {
            const float u = base[(long)y * m.sh + (long)x * m.sw];
            v = (u > v || u != u) ? u : v;  // NaN propagates like torch's max pooling
        }
    w[t] = v;
}

Map make_map(const float* p, const long* shape, const long* stride) {
    Map m;
    m.p = p;
    m.C = (int)shape[1];
    m.H = (int)shape[2];
    m.W = (int)shape[3];
    m.sb = stride[0];
    m.sc = stride[1];
    m.sh = stride[2];
    m.sw = stride[3];
    return m;
}

}  // namespace

extern "C" long fpm_feature_align_ws_floats(const long* node_shape, const long* edge_shape) {
    return node_shape[0] * node_shape[2] * node_shape[3] + edge_shape[0] * edge_shape[2] * edge_shape[3];
}

extern "C" int fpm_feature_align_fwd(const float* nodes, const long* node_shape, const long* node_stride,
                                     const float* edges, const long* edge_shape, const long* edge_stride,
                                     const float* P, const int* n, int nmax, float ori_w, float ori_h, float* ws,
                                     float* X, long ldx, float* wglob, void* stream) {
    FPM_CHECK_ARG(node_shape[0] == edge_shape[0], "feature_align: node/edge maps disagree on the batch size");
    FPM_CHECK_ARG(node_shape[2] > 0 && node_shape[3] > 0 && edge_shape[2] > 0 && edge_shape[3] > 0,
                  "feature_align: empty feature map");
    FPM_CHECK_ARG(ldx >= node_shape[1] + edge_shape[1], "feature_align: ldx < C_nodes + C_edges");
    const int B = (int)node_shape[0];
    if (B == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const Map mn = make_map(nodes, node_shape, node_stride);
    const Map me = make_map(edges, edge_shape, edge_stride);
    float* nn_ = ws;
    float* ne_ = ws + (long)B * mn.H * mn.W;
    const long pn = (long)B * mn.H * mn.W, pe = (long)B * me.H * me.W;
    hipLaunchKernelGGL(pixel_norm_kernel, dim3((unsigned)((pn + 3) / 4)), dim3(256), 0, st, mn, B, nn_);
    hipLaunchKernelGGL(pixel_norm_kernel, dim3((unsigned)((pe + 3) / 4)), dim3(256), 0, st, me, B, ne_);
    if (nmax > 0)
        hipLaunchKernelGGL(feature_align_kernel, dim3((unsigned)(((long)B * nmax + 3) / 4)), dim3(256), 0, st, mn, me,
                           nn_, ne_, P, n, B, nmax, ori_w, ori_h, X, ldx);
    if (wglob)
        hipLaunchKernelGGL(global_maxpool_kernel, dim3((unsigned)(((long)B * me.C + 255) / 256)), dim3(256), 0, st,
                           me, B, wglob);
    return fpm::check_launch("fpm_feature_align_fwd");
}
