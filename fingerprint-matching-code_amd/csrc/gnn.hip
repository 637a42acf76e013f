// Association-graph GNN layer (reference PYGNNLayer.forward, src/model/gnn.py:207-226, over the
// sparse Kronecker pattern built at ngm.py:326-344) without materialising the pattern.
//
// torch_sparse mean aggregation over {Kronecker edge pairs} U {diagonal} factorises exactly:
//   agg[c][d][i] = ( sum_{a in N1(i)} sum_{e in N2(d)} X[c][e][a] + D[d][i] X[c][d][i] )
//                  / ( deg1(i) deg2(d) + D[d][i] ),   D = [d*n1max + i < n1b*n2b]  (quirk A.10(ii))
// Layout: X[b][c][d][i] (channel-major, i = graph-1 node fastest), p(i,d) = d*n1max + i.
//
// Work split.  One workgroup per (pair, graph-2 node d), one thread per graph-1 node i.  Phase 1
// sums the rows X[c][e][:] of d's graph-2 neighbours e (coalesced along i, two rows' loads in
// flight, the neighbour ids read with scalar loads straight from the CSR) into LDS, node-major;
// phase 2 gathers i's graph-1 neighbours from there and runs the node MLPs on packed fp32 FMAs:
//   x1 = lin_l(agg) + lin_r(x) + relu(W2 relu(W1 x + b1) + b2),  z = classifier(x1).
// (An fp32-MFMA variant of the MLPs measured slower: fp32 MFMA has the packed-FMA rate on CDNA4.)
// Block order: all blocks of a pair run on ONE XCD (workgroups are dealt to the 8 XCDs round-robin
// by linear id), so the pair's slab is re-read from that XCD's L2.  (Measured and dropped: a
// breadth-first block order of graph 2, -2 % per layer for a 0.1 ms order kernel per chunk, and
// workgroups of 2-4 BFS-consecutive nodes loading their neighbour-row union once: the larger
// workgroups lost more to occupancy than the shared loads saved.)
#include "fpm_common.h"
#include <cstdlib>

namespace {

// linear block id -> (pair b, graph-2 node d): XCD x = id % 8 takes pairs x, x+8, ... in d order
__device__ __forceinline__ bool pair_block(int n2max, int B, int& b, int& d) {
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    b = (k / n2max) * 8 + x;
    d = k % n2max;
    return b < B;
}

inline unsigned pair_grid(int n2max, int B) { return (unsigned)(((B + 7) / 8) * 8 * n2max); }

// packed per-layer parameters (f32), weights TRANSPOSED so output channels o, o+1 are adjacent
// (one 64-bit scalar operand of v_pk_fma_f32): WlT[C][16] bl[16] WrT[C][16] W1T[C][16] b1[16]
// W2T[16 (m)][16 (o)] b2[16] wc[16] bc; every block offset is even (8-B aligned pairs)
template <int C>
struct GnnPack {
    static constexpr int Wl = 0, bl = Wl + 16 * C, Wr = bl + 16, W1 = Wr + 16 * C, b1 = W1 + 16 * C, W2 = b1 + 16,
                         b2 = W2 + 256, wc = b2 + 16, bc = wc + 16, total = bc + 1;
};

typedef float f2_t __attribute__((ext_vector_type(2)));

// acc += w * (v.lo, v.lo) (hi = false) or w * (v.hi, v.hi): one v_pk_fma_f32, w a scalar pair
__device__ __forceinline__ void pk_fma_bcast(f2_t& acc, f2_t w, f2_t v, bool hi) {
    if (hi) asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(w), "v"(v));
    else asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "s"(w), "v"(v));
}

// Phase 2 of one association node p = (d, i): agg from the graph-2 sums in LDS (Tg, node-major,
// TS floats per graph-1 node) gathered over i's graph-1 neighbours, the mean, the node MLPs and
// classifier (output channels in pairs (o, o+1) on v_pk_fma_f32: the same fma chain per channel as
// scalar FMAs, half the VALU instructions; the weight pair is one 64-bit scalar operand, the input
// broadcast from one half of a VGPR pair by op_sel), then the stores.
template <int C, int TS, int SPOL = 0, bool MLP = true>
__device__ __forceinline__ void gnn_point(const float* Tg, __amdgpu_buffer_rsrc_t xr, int N4, long N, int n1max,
                                          int b, int d, int i, int nn2, const int* __restrict__ ptr1,
                                          const int* __restrict__ nbr1, int n1b, int n2b, const float* __restrict__ W,
                                          float* __restrict__ Xo, float* __restrict__ zbuf, float* __restrict__ vpart,
                                          const float* __restrict__ cls_w) {
    using P = GnnPack<C>;
    const long p = (long)d * n1max + i;
    // the pair's 17 output channels as one buffer resource: channel o at SGPR offset o * N4
    const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc((void*)(Xo + (long)b * 17 * N), (short)0,
                                                                         (int)(17 * N * 4), 0x00020000);
    // SPOL: the stores' cache policy (16 = sc1: the written lines leave the XCD's L2 instead of
    // evicting the pair's input slab, which the other blocks of the pair are still reading; the
    // next layer reads this output long after it has left L2 either way)
    auto store_o = [&](int o, float v) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orr, (int)p * 4, o * N4, SPOL);
    };
    const int beg = ptr1[(long)b * n1max + i], end = ptr1[(long)b * n1max + i + 1];
    const bool self = p < (long)n1b * n2b;
    float x[C], agg[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        x[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (int)p * 4, c * N4, 0));
        agg[c] = 0.f;
    }
    for (int e = beg; e < end; ++e) {
        const float* Ta = Tg + nbr1[e] * TS;
        if constexpr (C == 17) {
            static_assert(TS % 4 == 0, "16-B aligned node rows");
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 t4 = *(const float4*)(Ta + 4 * q);
                agg[4 * q] += t4.x;
                agg[4 * q + 1] += t4.y;
                agg[4 * q + 2] += t4.z;
                agg[4 * q + 3] += t4.w;
            }
            agg[16] += Ta[16];
        } else {
            agg[0] += Ta[0];
        }
    }
    const float cnt = (float)((end - beg) * nn2 + (self ? 1 : 0));
    // one division per position, C multiplies (within 1 ulp of the per-channel v / cnt; the C IEEE
    // divisions were ~12 % of the layer's VALU instructions)
    const float rc = cnt > 0.f ? 1.f / cnt : 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        float v = self ? agg[c] + x[c] : agg[c];
        agg[c] = v * rc;
    }
    if constexpr (!MLP) {
        // timing probe only (fpm_set_tuning("gnn_mlp_off", 1)): the aggregation, reads and stores
        // of the layer without the node MLPs -- NOT the layer's result
#pragma unroll
        for (int o = 0; o < 16; ++o) store_o(o, agg[o % C] + x[o % C]);
        zbuf[(long)b * N + p] = agg[0];
        return;
    }
    constexpr int CP = (C + 1) / 2;
    f2_t x2[CP], a2[CP];
#pragma unroll
    for (int k = 0; k < CP; ++k) {
        x2[k] = (f2_t){x[2 * k], 2 * k + 1 < C ? x[2 * k + 1] : 0.f};
        a2[k] = (f2_t){agg[2 * k], 2 * k + 1 < C ? agg[2 * k + 1] : 0.f};
    }
    const f2_t* W2p = (const f2_t*)W;                     // pair view (all block offsets even)
    f2_t h[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        f2_t s = W2p[(P::b1 >> 1) + m];
#pragma unroll
        for (int c = 0; c < C; ++c) pk_fma_bcast(s, W2p[((P::W1 + c * 16) >> 1) + m], x2[c >> 1], c & 1);
        h[m] = (f2_t){fmaxf(s.x, 0.f), fmaxf(s.y, 0.f)};
    }
    float z = 0.f, vp = 0.f;
#pragma unroll
    for (int op = 0; op < 8; ++op) {
        const int o = 2 * op;
        f2_t l = {0.f, 0.f}, r = {0.f, 0.f}, t = {0.f, 0.f};
#pragma unroll
        for (int c = 0; c < C; ++c) {
            pk_fma_bcast(l, W2p[((P::Wl + c * 16) >> 1) + op], a2[c >> 1], c & 1);
            pk_fma_bcast(r, W2p[((P::Wr + c * 16) >> 1) + op], x2[c >> 1], c & 1);
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) pk_fma_bcast(t, W2p[((P::W2 + m * 16) >> 1) + op], h[m >> 1], m & 1);
        const f2_t tb = t + W2p[(P::b2 >> 1) + op];
        const f2_t x1 = ((l + W2p[(P::bl >> 1) + op]) + r) + (f2_t){fmaxf(tb.x, 0.f), fmaxf(tb.y, 0.f)};
        if (vpart) {
            vp = fmaf(cls_w[o], x1.x, vp);
            vp = fmaf(cls_w[o + 1], x1.y, vp);
        } else {
            store_o(o, x1.x);
            store_o(o + 1, x1.y);
        }
        z = fmaf(W[P::wc + o], x1.x, z);
        z = fmaf(W[P::wc + o + 1], x1.y, z);
    }
    if (vpart) vpart[(long)b * N + p] = vp;
    zbuf[(long)b * N + p] = z + W[P::bc];
}

// NSW > 1 (C = 17): phase 1 sweeps the neighbour rows once per channel group (NSW groups) instead
// of once for all 17 channels -- the blocks of a pair run in step, so the pair's slab resident in the
// XCD's L2 at a time is one group's share (4.46 MB / NSW at n = 256) instead of the whole slab; the
// per-channel sums keep the neighbour-list order (bit-identical)
template <int C, int SPOL = 0, bool MLP = true, int NSW = 1>
__global__ __launch_bounds__(1024) void gnn_layer_kernel(const float* __restrict__ X, int n1max, int n2max,
                                                         const int* __restrict__ ptr1, const int* __restrict__ nbr1,
                                                         const int* __restrict__ ptr2, const int* __restrict__ nbr2,
                                                         const int* __restrict__ n1,
                                                         const int* __restrict__ n2, const float* __restrict__ W,
                                                         float* __restrict__ Xo, float* __restrict__ zbuf,
                                                         float* __restrict__ vpart, const float* __restrict__ cls_w,
                                                         int B, const int* __restrict__ ord2) {
    // T[i][TS]: sum of graph-2 neighbour rows, node-major with 80-B rows (C = 17) so phase 2
    // reads a neighbour's 17 channels with 4 ds_read_b128 + 1 ds_read_b32
    constexpr int TS = C == 1 ? 1 : 20;
    extern __shared__ __attribute__((aligned(16))) float T[];
    int b, d;
    if (!pair_block(n2max, B, b, d)) return;
    // ord2 (optional): the k-th block of a pair takes graph-2 node ord2[b][k] -- a schedule only (each
    // node's work is unchanged), so that the blocks in flight share neighbour rows in L2
    if (ord2) d = ord2[(long)b * n2max + d];
    const int i = threadIdx.x;
    const long N = (long)n1max * n2max;
    const float* Xb = X + (long)b * C * N;
    // the pair's C channels as one buffer resource (host check: 17 * N * 4 < 2^31)
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)Xb, (short)0, (int)(C * N * 4), 0x00020000);
    const int N4 = (int)(N * 4);
    const int beg2 = ptr2[(long)b * n2max + d], end2 = ptr2[(long)b * n2max + d + 1];
    if (i < n1max) {
        float acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.f;
        // buffer loads: one 32-bit VGPR row offset + the channel as an SGPR offset; the neighbour
        // ids are uniform (scalar loads)
        auto load_row = [&](int r, float (&v)[C]) {
#pragma unroll
            for (int c = 0; c < C; ++c)
                v[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (r * n1max + i) * 4, c * N4, 0));
        };
        if constexpr (NSW == 1) {
            int k = beg2;
            for (; k + 1 < end2; k += 2) {          // two rows' loads in flight, summed in list order
                float va[C], vb[C];
                load_row(nbr2[k], va);
                load_row(nbr2[k + 1], vb);
#pragma unroll
                for (int c = 0; c < C; ++c) acc[c] += va[c];
#pragma unroll
                for (int c = 0; c < C; ++c) acc[c] += vb[c];
            }
            if (k < end2) {
                float va[C];
                load_row(nbr2[k], va);
#pragma unroll
                for (int c = 0; c < C; ++c) acc[c] += va[c];
            }
        } else {
            constexpr int GS = (C + NSW - 1) / NSW;   // channels per sweep
#pragma unroll
            for (int g0 = 0; g0 < C; g0 += GS) {
                int k = beg2;
                for (; k + 3 < end2; k += 4) {      // four rows' loads of the group in flight
                    float v[4][GS];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int r = nbr2[k + u];
#pragma unroll
                        for (int c = 0; c < GS; ++c)
                            if (g0 + c < C)
                                v[u][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (r * n1max + i) * 4,
                                                                                                (g0 + c) * N4, 0));
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int c = 0; c < GS; ++c)
                            if (g0 + c < C) acc[g0 + c] += v[u][c];
                }
                for (; k < end2; ++k) {
                    const int r = nbr2[k];
#pragma unroll
                    for (int c = 0; c < GS; ++c)
                        if (g0 + c < C)
                            acc[g0 + c] += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (r * n1max + i) * 4,
                                                                                                 (g0 + c) * N4, 0));
                }
            }
        }
        float* Ti = T + i * TS;
        if constexpr (C == 17) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *(float4*)(Ti + 4 * q) = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
            Ti[16] = acc[16];
        } else {
            Ti[0] = acc[0];
        }
    }
    __syncthreads();
    if (i >= n1max) return;
    gnn_point<C, TS, SPOL, MLP>(T, xr, N4, N, n1max, b, d, i, end2 - beg2, ptr1, nbr1, n1[b], n2[b], W, Xo, zbuf,
                                vpart, cls_w);
    (void)NSW;
}

// v[p] = classifier(emb[p]) (ngm.py:368), written as s[b][i][j] = v[b][j*n1max + i] (ngm.py:369).
// With vpart (the last GNN layer's w[0:16] . x1, fused there) only channel 16 (its Sinkhorn) is read.
// 64 x 64 (d, i) tiles transposed through LDS: reads along i and writes s along d are both
// coalesced (a per-(pair, d) form wrote each value to its own cache line).
__global__ __launch_bounds__(256) void node_classifier_t_kernel(const float* __restrict__ X, int n1max, int n2max,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bias,
                                                                const float* __restrict__ vpart,
                                                                float* __restrict__ s) {
    __shared__ float tile[64][65];                        // [i - i0][d - d0]
    const int b = blockIdx.z, d0 = blockIdx.y * 64, i0 = blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const long N = (long)n1max * n2max;
    const float* Xb = X + (long)b * 17 * N;
    const int i = i0 + tx;
#pragma unroll 4
    for (int r = 0; r < 16; ++r) {
        const int d = d0 + ty + 4 * r;
        if (d < n2max && i < n1max) {
            const long p = (long)d * n1max + i;
            float acc;
            if (vpart) {
                acc = fmaf(w[16], Xb[16L * N + p], vpart[(long)b * N + p]);
            } else {
                acc = 0.f;
#pragma unroll
                for (int c = 0; c < 17; ++c) acc += w[c] * Xb[(long)c * N + p];
            }
            tile[tx][ty + 4 * r] = acc + bias[0];
        }
    }
    __syncthreads();
    const int d = d0 + tx;
#pragma unroll 4
    for (int r = 0; r < 16; ++r) {
        const int ii = i0 + ty + 4 * r;
        if (ii < n1max && d < n2max) s[(long)b * N + (long)ii * n2max + d] = tile[ty + 4 * r][tx];
    }
}

}  // namespace

// fpm_set_tuning("gnn_store_sc1", v): the layer's output stores with the sc1 policy (1) or plain (0,
// default: measured neutral, 0.459 vs 0.462 ms per 17-channel launch alone, profiles/r04e_sc1_ab.txt)
// fpm_set_tuning("gnn_sweeps", 1 / 2 / 3): phase-1 channel-group sweeps of the 17-channel layer
int& gnn_sweeps_flag() {
    static int v = [] {
        const char* e = getenv("FPM_GNN_SWEEPS");
        return e ? atoi(e) : 1;
    }();
    return v;
}

int& gnn_store_sc1_flag() {
    static int v = [] {
        const char* e = getenv("FPM_GNN_SC1");
        return e ? atoi(e) : 0;
    }();
    return v;
}

// fpm_set_tuning("gnn_mlp_off", 1): timing probe -- the layer without its node MLPs (wrong results)
int& gnn_mlp_off_flag() {
    static int v = 0;
    return v;
}

extern "C" int fpm_kron_gnn_layer_fwd_ord(const float* X, int C, int B, int n1max, int n2max, const int* ptr1,
                                          const int* nbr1, const int* ptr2, const int* nbr2, const int* n1,
                                          const int* n2, const float* params, float* Xout, float* zbuf,
                                          float* vpart, const float* cls_w, const int* ord2, void* stream) {
    FPM_CHECK_ARG(C == 1 || C == 17, "gnn_layer: C must be 1 or 17 (got %d)", C);
    FPM_CHECK_ARG(!vpart || cls_w, "gnn_layer: vpart needs cls_w");
    if (B == 0) return 0;
    FPM_CHECK_ARG(n1max >= 1 && n1max <= 1024, "gnn_layer: n1max must be in [1, 1024]");
    FPM_CHECK_ARG((long)17 * n1max * n2max * 4 < (1L << 31), "gnn_layer: a pair's state must be < 2 GiB");
    const size_t sh = (size_t)(C == 1 ? 1 : 20) * n1max * 4;
    const int threads = (n1max + 63) / 64 * 64;
    void (*k)(const float*, int, int, const int*, const int*, const int*, const int*, const int*, const int*,
              const float*, float*, float*, float*, const float*, int, const int*) =
        (C == 17 && gnn_sweeps_flag() == 2 && !gnn_mlp_off_flag() && !gnn_store_sc1_flag()) ? gnn_layer_kernel<17, 0, true, 2>
        : (C == 17 && gnn_sweeps_flag() == 3 && !gnn_mlp_off_flag() && !gnn_store_sc1_flag()) ? gnn_layer_kernel<17, 0, true, 3>
        : gnn_mlp_off_flag() ? (C == 1 ? gnn_layer_kernel<1, 0, false> : gnn_layer_kernel<17, 0, false>)
        : gnn_store_sc1_flag() ? (C == 1 ? gnn_layer_kernel<1, 16> : gnn_layer_kernel<17, 16>)
                               : (C == 1 ? gnn_layer_kernel<1> : gnn_layer_kernel<17>);
    if (sh > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    hipLaunchKernelGGL(k, dim3(pair_grid(n2max, B)), dim3(threads), sh, (hipStream_t)stream, X, n1max, n2max, ptr1,
                       nbr1, ptr2, nbr2, n1, n2, params, Xout, zbuf, vpart, cls_w, B, ord2);
    return fpm::check_launch("fpm_kron_gnn_layer_fwd");
}

extern "C" int fpm_kron_gnn_layer_fwd(const float* X, int C, int B, int n1max, int n2max, const int* ptr1,
                                      const int* nbr1, const int* ptr2, const int* nbr2, const int* n1,
                                      const int* n2, const float* params, float* Xout, float* zbuf,
                                      float* vpart, const float* cls_w, void* stream) {
    return fpm_kron_gnn_layer_fwd_ord(X, C, B, n1max, n2max, ptr1, nbr1, ptr2, nbr2, n1, n2, params, Xout, zbuf,
                                      vpart, cls_w, nullptr, stream);
}

extern "C" int fpm_gnn_param_count(int C) { return C == 1 ? GnnPack<1>::total : GnnPack<17>::total; }

extern "C" int fpm_node_classifier(const float* X, int B, int n1max, int n2max, const float* w, const float* bias,
                                   const float* vpart, float* s, void* stream) {
    if (B == 0) return 0;
    FPM_CHECK_ARG(B <= 65535, "node_classifier: B must be <= 65535");
    const dim3 grid((unsigned)((n1max + 63) / 64), (unsigned)((n2max + 63) / 64), (unsigned)B);
    hipLaunchKernelGGL(node_classifier_t_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, n1max, n2max, w, bias,
                       vpart, s);
    return fpm::check_launch("fpm_node_classifier");
}

// ---- training backward -------------------------------------------------
// The factorised SAGE-mean aggregation alone (no MLPs), in two directions:
//   adj = 0:  out[c][d][i] = ( sum_{a in T1(i)} sum_{e in T2(d)} X[c][e][a] + D[d][i] X[c][d][i] ) / den[d][i]
//   adj = 1:  the same traversal of Xs = X / den (0 where den = 0) without the final division,
// where den[d][i] = deg1(i) deg2(d) + D[d][i] with in-degrees from (q1, q2).  With (T1, T2) the
// in-edge CSRs, adj = 0 recomputes the forward's agg (gnn_layer_kernel); with the OUT-edge CSRs
// (the plans of the reversed edge lists), adj = 1 is its transpose, the gradient path
// dX = A1^T G A2 + D o G, G = dagg / den.  One workgroup per (pair, graph-2 node), one thread per
// graph-1 node, the graph-2 neighbour sums staged in LDS [c][n1max].
namespace {
__global__ __launch_bounds__(1024) void kron_agg_kernel(const float* __restrict__ X, int C, int n1max, int n2max,
                                                        const int* __restrict__ tptr1, const int* __restrict__ tnbr1,
                                                        const int* __restrict__ tptr2, const int* __restrict__ tnbr2,
                                                        const int* __restrict__ q1, const int* __restrict__ q2,
                                                        const int* __restrict__ n1, const int* __restrict__ n2,
                                                        int adj_flags, float* __restrict__ out, int B) {
    extern __shared__ float T[];
    int d, b;
    if (!pair_block(n2max, B, b, d)) return;
    const int adj = adj_flags & 1;
    const bool accum = (adj_flags & 2) != 0;
    const int i = threadIdx.x;
    const long N = (long)n1max * n2max;
    const float* Xb = X + (long)b * C * N;
    const long nb1 = (long)b * n1max, nb2 = (long)b * n2max;
    const long nn = (long)n1[b] * n2[b];
    auto den = [&](int dd, int ii) -> float {
        const int g1 = q1[nb1 + ii + 1] - q1[nb1 + ii];
        const int g2 = q2[nb2 + dd + 1] - q2[nb2 + dd];
        return (float)(g1 * g2 + (((long)dd * n1max + ii) < nn ? 1 : 0));
    };
    auto xval = [&](int c, int dd, int ii) -> float {
        const float x = Xb[(long)c * N + (long)dd * n1max + ii];
        if (!adj) return x;
        const float dn = den(dd, ii);
        return dn > 0.f ? x / dn : 0.f;
    };
    if (i < n1max) {
        const int beg = tptr2[nb2 + d], end = tptr2[nb2 + d + 1];
        for (int c = 0; c < C; ++c) {
            float acc = 0.f;
            for (int e = beg; e < end; ++e) acc += xval(c, tnbr2[e], i);
            T[c * n1max + i] = acc;
        }
    }
    __syncthreads();
    if (i >= n1max) return;
    const int beg = tptr1[nb1 + i], end = tptr1[nb1 + i + 1];
    const bool self = ((long)d * n1max + i) < nn;
    const float dn = adj ? 1.f : den(d, i);
    for (int c = 0; c < C; ++c) {
        float acc = 0.f;
        for (int e = beg; e < end; ++e) acc += T[c * n1max + tnbr1[e]];
        if (self) acc += xval(c, d, i);
        float* o = out + (long)b * C * N + (long)c * N + (long)d * n1max + i;
        const float r = adj ? acc : (dn > 0.f ? acc / dn : 0.f);
        *o = accum ? *o + r : r;
    }
}
// The same for C = 1 / 17 with the channel loops unrolled (C independent loads per neighbour row in
// flight instead of a dependent per-channel loop) and the adjoint's per-element 1 / den(dd, i)
// computed once per (neighbour, thread) from the thread's graph-1 degree and the neighbour's
// graph-2 degree (multiplied, not divided: the gradient path has no bitwise contract).
template <int C>
__global__ __launch_bounds__(1024) void kron_agg_c_kernel(const float* __restrict__ X, int n1max, int n2max,
                                                          const int* __restrict__ tptr1, const int* __restrict__ tnbr1,
                                                          const int* __restrict__ tptr2, const int* __restrict__ tnbr2,
                                                          const int* __restrict__ q1, const int* __restrict__ q2,
                                                          const int* __restrict__ n1, const int* __restrict__ n2,
                                                          int adj_flags, float* __restrict__ out, int B) {
    extern __shared__ float T[];                           // [i][C] node-major
    int d, b;
    if (!pair_block(n2max, B, b, d)) return;
    const int adj = adj_flags & 1;
    const bool accum = (adj_flags & 2) != 0;
    const int i = threadIdx.x;
    const long N = (long)n1max * n2max;
    const float* Xb = X + (long)b * C * N;
    const long nb1 = (long)b * n1max, nb2 = (long)b * n2max;
    const long nn = (long)n1[b] * n2[b];
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)Xb, (short)0, (int)(C * N * 4), 0x00020000);
    const int N4 = (int)(N * 4);
    const int g1 = i < n1max ? q1[nb1 + i + 1] - q1[nb1 + i] : 0;
    if (i < n1max) {
        const int beg = tptr2[nb2 + d], end = tptr2[nb2 + d + 1];
        float acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.f;
        for (int e = beg; e < end; ++e) {
            const int dd = tnbr2[e];
            float sc = 1.f;
            if (adj) {
                const int g2 = q2[nb2 + dd + 1] - q2[nb2 + dd];
                const float dn = (float)(g1 * g2 + (((long)dd * n1max + i) < nn ? 1 : 0));
                sc = dn > 0.f ? 1.f / dn : 0.f;
            }
            const int off = (dd * n1max + i) * 4;
            float v[C];
#pragma unroll
            for (int c = 0; c < C; ++c) v[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off, c * N4, 0));
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = fmaf(v[c], sc, acc[c]);
        }
#pragma unroll
        for (int c = 0; c < C; ++c) T[i * C + c] = acc[c];
    }
    __syncthreads();
    if (i >= n1max) return;
    const int beg = tptr1[nb1 + i], end = tptr1[nb1 + i + 1];
    const long pos = (long)d * n1max + i;
    const bool self = pos < nn;
    const int g2d = q2[nb2 + d + 1] - q2[nb2 + d];
    const float dn = (float)(g1 * g2d + (self ? 1 : 0));
    const float rdn = dn > 0.f ? 1.f / dn : 0.f;
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = 0.f;
    for (int e = beg; e < end; ++e) {
        const float* Ta = T + tnbr1[e] * C;
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] += Ta[c];
    }
    const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc((void*)(out + (long)b * C * N), (short)0,
                                                                         (int)(C * N * 4), 0x00020000);
#pragma unroll
    for (int c = 0; c < C; ++c) {
        float a = acc[c];
        if (self) {
            const float x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (int)pos * 4, c * N4, 0));
            a += adj ? x * rdn : x;
        }
        float r = adj ? a : a * rdn;
        if (accum) r += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(orr, (int)pos * 4, c * N4, 0));
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r), orr, (int)pos * 4, c * N4, 0);
    }
}
}  // namespace

extern "C" int fpm_kron_agg(const float* X, int C, int B, int n1max, int n2max, const int* tptr1, const int* tnbr1,
                            const int* tptr2, const int* tnbr2, const int* q1, const int* q2, const int* n1,
                            const int* n2, int adjoint, float* out, void* stream) {
    FPM_CHECK_ARG(C >= 1 && C <= 32, "kron_agg: C must be in [1, 32]");
    FPM_CHECK_ARG(n1max <= 1024, "kron_agg: n1max must be <= 1024");
    if (B == 0) return 0;
    const size_t sh = (size_t)C * n1max * sizeof(float);
    if (sh > 65536)
        (void)hipFuncSetAttribute((const void*)kron_agg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    const int threads = (n1max + 63) / 64 * 64;
    if ((C == 1 || C == 17) && (long)C * n1max * n2max * 4 < (1L << 31)) {
        void (*k)(const float*, int, int, const int*, const int*, const int*, const int*, const int*, const int*,
                  const int*, const int*, int, float*, int) = C == 1 ? kron_agg_c_kernel<1> : kron_agg_c_kernel<17>;
        if (sh > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        hipLaunchKernelGGL(k, dim3(pair_grid(n2max, B)), dim3(threads), sh, (hipStream_t)stream, X, n1max, n2max, tptr1,
                           tnbr1, tptr2, tnbr2, q1, q2, n1, n2, adjoint, out, B);
        return fpm::check_launch("fpm_kron_agg");
    }
    hipLaunchKernelGGL(kron_agg_kernel, dim3(pair_grid(n2max, B)), dim3(threads), sh, (hipStream_t)stream, X, C, n1max,
                       n2max, tptr1, tnbr1, tptr2, tnbr2, q1, q2, n1, n2, adjoint, out, B);
    return fpm::check_launch("fpm_kron_agg");
}

// Per-position part of the PYGNNLayer backward (the node MLPs of gnn_layer_kernel, transposed):
// with dx1 = dXn[0:16] + wc * dz (classifier), recompute h1 = relu(W1 x + b1), h2 = W2 h1 + b2,
//   dm = dx1 o [h2 > 0],  dh1 = (W2^T dm) o [h1 > 0],
//   dX = W1^T dh1 + Wr^T dx1 (the direct part; the aggregation part is fpm_kron_agg's adjoint
//   of dagg),  dagg = Wl^T dx1,
// and store the per-position vectors the weight gradients reduce over: V[b] = [dx1 | dh1 | dm | h1]
// (4 x 16 channels, channel-major).  One thread per (pair, position); uniform weights in SGPRs.
namespace {
template <int C>
__global__ __launch_bounds__(256) void gnn_bwd_point_kernel(const float* __restrict__ X, const float* __restrict__ dXn,
                                                            const float* __restrict__ dz, const float* __restrict__ W,
                                                            int B, long N, float* __restrict__ dX,
                                                            float* __restrict__ dagg, float* __restrict__ V) {
    using P = GnnPack<C>;
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    if (t >= (long)B * N) return;
    const long b = t / N, p = t - b * N;
    const float* Xb = X + b * C * N + p;
    const float* Gb = dXn + b * 17 * N + p;
    float x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = Xb[(long)c * N];
    const float g = dz[b * N + p];
    float dx1[16], h1[16], dm[16];
    float h1p[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        float s = W[P::b1 + m];
#pragma unroll
        for (int c = 0; c < C; ++c) s += W[P::W1 + c * 16 + m] * x[c];
        h1p[m] = s;
        h1[m] = fmaxf(s, 0.f);
    }
#pragma unroll
    for (int o = 0; o < 16; ++o) {
        dx1[o] = Gb[(long)o * N] + W[P::wc + o] * g;
        float s = W[P::b2 + o];
#pragma unroll
        for (int m = 0; m < 16; ++m) s += W[P::W2 + m * 16 + o] * h1[m];
        dm[o] = s > 0.f ? dx1[o] : 0.f;
    }
    float* Vb = V + b * 64 * N + p;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        float s = 0.f;
#pragma unroll
        for (int o = 0; o < 16; ++o) s += W[P::W2 + m * 16 + o] * dm[o];
        const float dh = h1p[m] > 0.f ? s : 0.f;
        Vb[(long)(16 + m) * N] = dh;
        h1p[m] = dh;      // reuse as dh1
    }
#pragma unroll
    for (int o = 0; o < 16; ++o) {
        Vb[(long)o * N] = dx1[o];
        Vb[(long)(32 + o) * N] = dm[o];
        Vb[(long)(48 + o) * N] = h1[o];
    }
    float* dXb = dX + b * C * N + p;
    float* dAb = dagg + b * C * N + p;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        float s = 0.f, r = 0.f;
#pragma unroll
        for (int m = 0; m < 16; ++m) s += W[P::W1 + c * 16 + m] * h1p[m];
#pragma unroll
        for (int o = 0; o < 16; ++o) {
            s += W[P::Wr + c * 16 + o] * dx1[o];
            r += W[P::Wl + c * 16 + o] * dx1[o];
        }
        dXb[(long)c * N] = s;
        dAb[(long)c * N] = r;
    }
}
}  // namespace

extern "C" int fpm_kron_gnn_layer_bwd_point(const float* X, int C, int B, int n1max, int n2max, const float* dXn,
                                            const float* dz, const float* params, float* dX, float* dagg, float* V,
                                            void* stream) {
    FPM_CHECK_ARG(C == 1 || C == 17, "gnn_layer_bwd: C must be 1 or 17 (got %d)", C);
    if (B == 0) return 0;
    const long N = (long)n1max * n2max;
    const unsigned grid = (unsigned)(((long)B * N + 255) / 256);
    hipStream_t st = (hipStream_t)stream;
    if (C == 1)
        hipLaunchKernelGGL((gnn_bwd_point_kernel<1>), dim3(grid), dim3(256), 0, st, X, dXn, dz, params, B, N, dX, dagg, V);
    else
        hipLaunchKernelGGL((gnn_bwd_point_kernel<17>), dim3(grid), dim3(256), 0, st, X, dXn, dz, params, B, N, dX, dagg,
                           V);
    return fpm::check_launch("fpm_kron_gnn_layer_bwd_point");
}
