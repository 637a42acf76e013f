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

// ---- backward (train.py stages 1 / 3 / 5 train the backbone through this stage) ----------------
// Per map and image pixel, one workgroup: the keypoints whose bilinear corners hit the pixel are
// found by recomputing every keypoint's corners exactly as the forward does (fixed keypoint order,
// a pixel's weights of one keypoint summed over its corners q = a, b, c, d), then
//   dy[c]  = sum_i w_i(pixel) * dX[i][off + c]                 (transpose of the gather)
//   dx[c]  = (dy[c] - y[c] * sum_c' y[c'] dy[c']) / |x|        (y = x / |x|, normalize_over_channels)
// written once per (image, channel, pixel) -- no atomics.  The global max-pool's gradient is added
// afterwards by global_maxpool_bwd_kernel at each (image, channel)'s first maximum (torch's
// AdaptiveMaxPool2d index rule, NaN last-wins like the forward).
constexpr int FB_T = 256;

__global__ __launch_bounds__(FB_T) void feature_align_bwd_kernel(Map m, Map g, const float* __restrict__ nrm,
                                                                 const float* __restrict__ P,
                                                                 const int* __restrict__ nv, int nmax, float ox,
                                                                 float oy, const float* __restrict__ dX, long ldx,
                                                                 int coff) {
    extern __shared__ float wl[];                 // nmax weights, then the compact hit list
    __shared__ float red[FB_T / 64];
    __shared__ int nhit;
    const int HW = m.H * m.W;
    const long b = blockIdx.x / HW;
    const int pix = (int)(blockIdx.x - b * HW);
    const int tid = threadIdx.x, lane = tid & 63;
    const int n = nv[b];
    for (int i = tid; i < n; i += FB_T) {
        float x, y;
        to_map(P[(b * nmax + i) * 2], P[(b * nmax + i) * 2 + 1], ox, oy, m.H, m.W, x, y);
        const Corner c = corners(x, y, m.H, m.W);
        float w = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (c.off[q] == pix) w += c.w[q];
        // hits are flagged by the corner test, not by w != 0 (a zero weight still indexes the pixel)
        bool hit = c.off[0] == pix || c.off[1] == pix || c.off[2] == pix || c.off[3] == pix;
        wl[i] = hit ? w : __int_as_float(0x7fc00001);   // a NaN payload marks "no hit"
    }
    __syncthreads();
    // compact (keypoint, weight) pairs in ascending keypoint order (wave 0)
    int* hid = (int*)(wl + nmax);
    float* hw = (float*)(hid + nmax);
    if (tid < 64) {
        int cnt = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            const float w = i < n ? wl[i] : 0.f;
            const bool h = i < n && __float_as_int(w) != 0x7fc00001;
            const unsigned long long bal = __ballot(h);
            if (h) {
                const int slot = cnt + __popcll(bal & ((1ull << lane) - 1ull));
                hid[slot] = i;
                hw[slot] = w;
            }
            cnt += __popcll(bal);
        }
        if (lane == 0) nhit = cnt;
    }
    __syncthreads();
    const int nh = nhit;
    const float inv = 1.f / nrm[b * HW + pix];
    const int yy = pix / m.W, xx = pix - yy * m.W;
    const float* xp = m.p + b * m.sb + (long)yy * m.sh + (long)xx * m.sw;
    float* gp = (float*)g.p + b * g.sb + (long)yy * g.sh + (long)xx * g.sw;
    constexpr int CPT = 2;                       // channels per thread (C <= 512)
    float dy[CPT], yv[CPT];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const int ch = tid + k * FB_T;
        dy[k] = 0.f;
        yv[k] = 0.f;
        if (ch < m.C) {
            float a = 0.f;
            for (int h = 0; h < nh; ++h) a = fmaf(hw[h], dX[(b * nmax + hid[h]) * ldx + coff + ch], a);
            dy[k] = a;
            yv[k] = xp[(long)ch * m.sc] * inv;
            dot = fmaf(yv[k], a, dot);
        }
    }
    dot = fpm::warp_sum(dot);
    if (lane == 0) red[tid >> 6] = dot;
    __syncthreads();
    dot = 0.f;
#pragma unroll
    for (int w = 0; w < FB_T / 64; ++w) dot += red[w];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const int ch = tid + k * FB_T;
        if (ch < m.C) gp[(long)ch * g.sc] = (dy[k] - yv[k] * dot) * inv;
    }
}

__global__ void global_maxpool_bwd_kernel(Map m, Map g, int B, const float* __restrict__ dw) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B * m.C) return;
    const long b = t / m.C;
    const int c = (int)(t - b * m.C);
    const float* base = m.p + b * m.sb + (long)c * m.sc;
    float v = -INFINITY;
    int arg = 0, k = 0;
    for (int y = 0; y < m.H; ++y)
        for (int x = 0; x < m.W; ++x, ++k) {
            const float u = base[(long)y * m.sh + (long)x * m.sw];
            if (u > v || u != u) {
                v = u;
                arg = k;
            }
        }
    const int y = arg / m.W, x = arg - (arg / m.W) * m.W;
    float* gp = (float*)g.p + b * g.sb + (long)c * g.sc + (long)y * g.sh + (long)x * g.sw;
    *gp += dw[t];
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

// Backward of fpm_feature_align_fwd: dX (B*nmax, ldx) and dwglob (B, C_edges, may be NULL) ->
// dnodes / dedges, gradients w.r.t. the raw CNN maps (same shapes; own strides).  ws: the forward's
// workspace (pixel norms, unchanged since the forward).  Every element of dnodes / dedges is written.
extern "C" int fpm_feature_align_bwd(const float* nodes, const long* node_shape, const long* node_stride,
                                     const float* edges, const long* edge_shape, const long* edge_stride,
                                     const float* P, const int* n, int nmax, float ori_w, float ori_h,
                                     const float* ws, const float* dX, long ldx, const float* dwglob, float* dnodes,
                                     const long* dnode_stride, float* dedges, const long* dedge_stride,
                                     void* stream) {
    FPM_CHECK_ARG(node_shape[0] == edge_shape[0], "feature_align_bwd: node/edge maps disagree on the batch size");
    FPM_CHECK_ARG(node_shape[1] <= 2 * FB_T && edge_shape[1] <= 2 * FB_T, "feature_align_bwd: at most %d channels",
                  2 * FB_T);
    FPM_CHECK_ARG(ldx >= node_shape[1] + edge_shape[1], "feature_align_bwd: ldx < C_nodes + C_edges");
    FPM_CHECK_ARG(nmax >= 0 && nmax <= 4096, "feature_align_bwd: nmax must be <= 4096");
    const int B = (int)node_shape[0];
    if (B == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const Map mn = make_map(nodes, node_shape, node_stride);
    const Map me = make_map(edges, edge_shape, edge_stride);
    const Map gn = make_map(dnodes, node_shape, dnode_stride);
    const Map ge = make_map(dedges, edge_shape, dedge_stride);
    const float* nn_ = ws;
    const float* ne_ = ws + (long)B * mn.H * mn.W;
    const size_t lds = (size_t)(nmax > 0 ? nmax : 1) * 3 * sizeof(float);
    hipLaunchKernelGGL(feature_align_bwd_kernel, dim3((unsigned)((long)B * mn.H * mn.W)), dim3(FB_T), lds, st, mn, gn,
                       nn_, P, n, nmax, ori_w, ori_h, dX, ldx, 0);
    hipLaunchKernelGGL(feature_align_bwd_kernel, dim3((unsigned)((long)B * me.H * me.W)), dim3(FB_T), lds, st, me, ge,
                       ne_, P, n, nmax, ori_w, ori_h, dX, ldx, mn.C);
    if (dwglob)
        hipLaunchKernelGGL(global_maxpool_bwd_kernel, dim3((unsigned)(((long)B * me.C + 255) / 256)), dim3(256), 0, st,
                           me, ge, B, dwglob);
    return fpm::check_launch("fpm_feature_align_bwd");
}
