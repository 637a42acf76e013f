// Association-graph GNN layer (reference PYGNNLayer.forward, src/model/gnn.py:207-226, over the
// sparse Kronecker pattern built at ngm.py:326-344) without materialising the pattern.
//
// torch_sparse mean aggregation over {Kronecker edge pairs} U {diagonal} factorises exactly:
//   agg[c][d][i] = ( sum_{a in N1(i)} sum_{b in N2(d)} X[c][b][a] + D[d][i] X[c][d][i] )
//                  / ( deg1(i) deg2(d) + D[d][i] ),   D = [d*n1max + i < n1b*n2b]  (quirk A.10(ii))
// One workgroup per (graph-2 node d, pair), one thread per graph-1 node i: the rows X[c][b][:] of
// d's neighbours are summed (coalesced) into LDS, then each thread gathers its i's graph-1
// neighbours from LDS and runs the node MLPs: x1 = lin_l(agg) + lin_r(x) + relu(W2 relu(W1 x + b1)
// + b2), z = classifier(x1).  (An fp32-MFMA variant of the MLPs measured slower: the layer is bound
// by the neighbour-row gathers, not the MLP arithmetic.)
// Layout: X[b][c][d][i] (channel-major, i = graph-1 node fastest), p(i,d) = d*n1max + i.
// Block order: all (d) blocks of a pair run on ONE XCD (workgroups are dealt to the 8 XCDs
// round-robin by linear id), so the pair's 17-channel slab (4.4 MB at n = 256) is re-read from
// that XCD's L2 by the ~6 neighbour blocks instead of from the fabric.
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

// WIDE (C = 17, n1max % 4 == 0): phase 1 with 16-B loads -- each thread sums one quad of graph-1
// positions (4 consecutive i) for a group of <= 5 channels, so a graph-2 neighbour row costs
// 17 / 4 times fewer vector-memory instructions; the per-position sums (same order, same
// values) land in the same LDS layout, so phase 2 and the outputs are bit-identical.
template <int C, bool PACKED, int U = 1, int G = 1, bool WIDE = false, bool IL = false>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(PACKED ? 5 : 6, 8))) void gnn_layer_kernel(const float* __restrict__ X, int n1max, int n2max,
                                                         const int* __restrict__ ptr1, const int* __restrict__ nbr1,
                                                         const int* __restrict__ ptr2, const int* __restrict__ nbr2,
                                                         const int* __restrict__ n1, const int* __restrict__ n2,
                                                         const float* __restrict__ W, float* __restrict__ Xo,
                                                         float* __restrict__ zbuf, float* __restrict__ vpart,
                                                         const float* __restrict__ cls_w, int B) {
    // one thread per graph-1 node i (blockDim >= n1max): no loop, so the uniform weight loads
    // stay scalar (s_load, SGPR operands of the FMAs) instead of being hoisted into VGPRs.
    using P = GnnPack<C>;
    // T[a][TS]: sum of graph-2 neighbour rows, node-major with 80-B rows (C = 17) so phase 2
    // reads a neighbour's 17 channels with 4 ds_read_b128 + 1 ds_read_b32
    constexpr int TS = C == 1 ? 1 : 20;
    extern __shared__ __attribute__((aligned(16))) float T[];
    __shared__ int nb2_[G][64];
    __shared__ int nnb2_[G], beg2_[G];

    // G > 1: G graph-2 nodes per workgroup, one thread group of blockDim / G each
    const int subw = G > 1 ? (int)blockDim.x / G : (int)blockDim.x;
    const int sub = G > 1 ? (int)threadIdx.x / subw : 0;
    const int i = G > 1 ? (int)threadIdx.x - sub * subw : (int)threadIdx.x;
    int dg, b;
    if (!pair_block((n2max + G - 1) / G, B, b, dg)) return;
    const int d = dg * G + sub;
    const bool active = d < n2max;
    int* nb2 = nb2_[sub];
    float* Tg = T + (long)sub * n1max * TS;
    const long N = (long)n1max * n2max;
    const float* Xb = X + (long)b * C * N;
    // the pair's C channels as one buffer resource (host check: C * N * 4 < 2^31)
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)Xb, (short)0, (int)(C * N * 4), 0x00020000);
    const int N4 = (int)(N * 4);
    if (i == 0 && active) {
        const int beg = ptr2[(long)b * n2max + d], end = ptr2[(long)b * n2max + d + 1];
        nnb2_[sub] = end - beg;
        beg2_[sub] = beg;
        for (int k = 0; k < end - beg && k < 64; ++k) nb2[k] = nbr2[beg + k];
    }
    __syncthreads();
    const int nn2 = active ? nnb2_[sub] : 0;
    const int beg2 = active ? beg2_[sub] : 0;
    if constexpr (WIDE) {
        static_assert(C == 17, "WIDE phase 1 is the 17-channel layer's");
        constexpr int CPG = 5;                               // ceil(17 / 4); ng >= 4 channel groups
        const int nq = n1max >> 2;
        const int ng = subw / nq;
        const int q = i % nq, g = i / nq;
        const int c0 = g * ((C + ng - 1) / ng);
        const int cn = min(C - c0, (C + ng - 1) / ng);
        if (active && g < ng && cn > 0) {
            float4 acc[CPG];
#pragma unroll
            for (int cc = 0; cc < CPG; ++cc) acc[cc] = make_float4(0.f, 0.f, 0.f, 0.f);
            const float* base = Xb + (long)c0 * N + 4 * q;
            auto add_row = [&](int nb) {
                const float* row = base + (long)nb * n1max;
                float4 v[CPG];
#pragma unroll
                for (int cc = 0; cc < CPG; ++cc)
                    if (cc < cn) v[cc] = *(const float4*)(row + (long)cc * N);
#pragma unroll
                for (int cc = 0; cc < CPG; ++cc)
                    if (cc < cn) {
                        acc[cc].x += v[cc].x;
                        acc[cc].y += v[cc].y;
                        acc[cc].z += v[cc].z;
                        acc[cc].w += v[cc].w;
                    }
            };
            const int nl = nn2 < 64 ? nn2 : 64;
            for (int k = 0; k < nl; ++k) add_row(nb2[k]);
            for (int k = 64; k < nn2; ++k) add_row(nbr2[beg2 + k]);
            float* Tq = Tg + 4 * q * TS + c0;
#pragma unroll
            for (int cc = 0; cc < CPG; ++cc)
                if (cc < cn) {
                    Tq[cc] = acc[cc].x;
                    Tq[TS + cc] = acc[cc].y;
                    Tq[2 * TS + cc] = acc[cc].z;
                    Tq[3 * TS + cc] = acc[cc].w;
                }
        }
    } else if (i < n1max && active) {
        // neighbour-outer, channel-inner: C independent loads in flight per neighbour row
        float acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.f;
        // buffer loads: one 32-bit VGPR row offset + the channel as an SGPR offset, instead of
        // 64-bit per-channel address math per load (~100 VALU per wave)
        auto add_row = [&](int nb) {
            const int off = (nb * n1max + i) * 4;
            float v[C];
#pragma unroll
            for (int c = 0; c < C; ++c) v[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off, c * N4, 0));
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] += v[c];
        };
        const int nl = nn2 < 64 ? nn2 : 64;
        int k0 = 0;
        if constexpr (U > 1) {
            // U neighbour rows' loads issued together (U x C in flight), summed in the same order
            for (; k0 + U <= nl; k0 += U) {
                float v[U][C];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const float* row = Xb + (long)nb2[k0 + u] * n1max + i;
#pragma unroll
                    for (int c = 0; c < C; ++c) v[u][c] = row[(long)c * N];
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int c = 0; c < C; ++c) acc[c] += v[u][c];
            }
        }
        for (int k = k0; k < nl; ++k) add_row(nb2[k]);                 // LDS copy of the first 64
        for (int k = 64; k < nn2; ++k) add_row(nbr2[beg2 + k]);

        float* Ti = Tg + i * TS;
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
    if (i >= n1max || !active) return;
    const int n1b = n1[b], n2b = n2[b];
    const long p = (long)d * n1max + i;
    // the pair's 17 output channels as one buffer resource: channel o at SGPR offset o * N4
    const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc((void*)(Xo + (long)b * 17 * N), (short)0,
                                                                         (int)(17 * N * 4), 0x00020000);
    auto store_o = [&](int o, float v) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orr, (int)p * 4, o * N4, 0);
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
    if (!PACKED) {
        float h[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            float s = W[P::b1 + m];
#pragma unroll
            for (int c = 0; c < C; ++c) s += W[P::W1 + c * 16 + m] * x[c];
            h[m] = fmaxf(s, 0.f);
        }
        float z = 0.f, vp = 0.f;
#pragma unroll
        for (int o = 0; o < 16; ++o) {
            float l = 0.f, r = 0.f, t = 0.f;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                l += W[P::Wl + c * 16 + o] * agg[c];
                r += W[P::Wr + c * 16 + o] * x[c];
            }
#pragma unroll
            for (int m = 0; m < 16; ++m) t += W[P::W2 + m * 16 + o] * h[m];
            float x1 = ((l + W[P::bl + o]) + r) + fmaxf(t + W[P::b2 + o], 0.f);
            if (vpart) vp = fmaf(cls_w[o], x1, vp);      // last layer: only w[0:16] . x1 is consumed
            else store_o(o, x1);
            z += W[P::wc + o] * x1;
        }
        if (vpart) vpart[(long)b * N + p] = vp;
        zbuf[(long)b * N + p] = z + W[P::bc];
        return;
    }
    // packed: output channels in pairs (o, o+1) on v_pk_fma_f32 -- the same fma chain per channel
    // as the scalar path (bit-identical), half the VALU instructions.  The weight pair is one
    // 64-bit scalar operand; the input value is broadcast from one half of a VGPR pair by op_sel.
    constexpr int CP = (C + 1) / 2;
    f2_t x2[CP], a2[CP];
#pragma unroll
    for (int k = 0; k < CP; ++k) {
        x2[k] = (f2_t){x[2 * k], 2 * k + 1 < C ? x[2 * k + 1] : 0.f};
        a2[k] = (f2_t){agg[2 * k], 2 * k + 1 < C ? agg[2 * k + 1] : 0.f};
    }
    const f2_t* W2p = (const f2_t*)W;                     // pair view (all block offsets even)
    if constexpr (IL) {
        // input-channel-outer order: a weight row W[c][0..15] is contiguous, so the scalar loads
        // merge into wide s_load_dwordx8/x16 (the per-(c, pair) order issued one s_load_dwordx2
        // per FMA: ~470 scalar-memory instructions per wave).  Every accumulator keeps its fma
        // chain order, so the outputs are bit-identical to the loop above.
        f2_t h[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) h[m] = W2p[(P::b1 >> 1) + m];
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int m = 0; m < 8; ++m) pk_fma_bcast(h[m], W2p[((P::W1 + c * 16) >> 1) + m], x2[c >> 1], c & 1);
#pragma unroll
        for (int m = 0; m < 8; ++m) h[m] = (f2_t){fmaxf(h[m].x, 0.f), fmaxf(h[m].y, 0.f)};
        float z = 0.f, vp = 0.f;
        constexpr int OPB = 4;                            // output pairs per block (register budget)
#pragma unroll
        for (int ob = 0; ob < 8; ob += OPB) {
            f2_t l[OPB], r[OPB], t[OPB];
#pragma unroll
            for (int k = 0; k < OPB; ++k) l[k] = r[k] = t[k] = (f2_t){0.f, 0.f};
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
                for (int k = 0; k < OPB; ++k) {
                    pk_fma_bcast(l[k], W2p[((P::Wl + c * 16) >> 1) + ob + k], a2[c >> 1], c & 1);
                    pk_fma_bcast(r[k], W2p[((P::Wr + c * 16) >> 1) + ob + k], x2[c >> 1], c & 1);
                }
#pragma unroll
            for (int m = 0; m < 16; ++m)
#pragma unroll
                for (int k = 0; k < OPB; ++k)
                    pk_fma_bcast(t[k], W2p[((P::W2 + m * 16) >> 1) + ob + k], h[m >> 1], m & 1);
#pragma unroll
            for (int k = 0; k < OPB; ++k) {
                const int op = ob + k, o = 2 * op;
                const f2_t tb = t[k] + W2p[(P::b2 >> 1) + op];
                const f2_t x1 = ((l[k] + W2p[(P::bl >> 1) + op]) + r[k]) + (f2_t){fmaxf(tb.x, 0.f), fmaxf(tb.y, 0.f)};
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
        }
        if (vpart) vpart[(long)b * N + p] = vp;
        zbuf[(long)b * N + p] = z + W[P::bc];
        return;
    }
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

// v[p] = classifier(emb[p]) (ngm.py:368), written as s[b][i][j] = v[b][j*n1max + i] (ngm.py:369).
// With vpart (the last GNN layer's w[0:16] . x1, fused there) only channel 16 (its Sinkhorn) is read.
__global__ __launch_bounds__(256) void node_classifier_kernel(const float* __restrict__ X, int n1max, int n2max,
                                                              const float* __restrict__ w, const float* __restrict__ bias,
                                                              const float* __restrict__ vpart, float* __restrict__ s,
                                                              int B) {
    int d, b;
    if (!pair_block(n2max, B, b, d)) return;
    const long N = (long)n1max * n2max;
    for (int i = threadIdx.x; i < n1max; i += 256) {
        const long p = (long)d * n1max + i;
        float acc;
        if (vpart) {
            acc = fmaf(w[16], X[(long)b * 17 * N + 16L * N + p], vpart[(long)b * N + p]);
        } else {
            acc = 0.f;
#pragma unroll
            for (int c = 0; c < 17; ++c) acc += w[c] * X[(long)b * 17 * N + (long)c * N + p];
        }
        s[(long)b * N + (long)i * n2max + d] = acc + bias[0];
    }
}

// The same on 64 x 64 (d, i) tiles transposed through LDS: reads along i and writes s along d are
// both coalesced (the per-(pair, d) form wrote each value to its own cache line, 4 B per lane at
// a 4 n2max-byte stride).  Same arithmetic per element, bit-identical.
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

// node classifier through the LDS transpose (1, default) or the per-(pair, d) form (0);
// env FPM_NODECLS_T or fpm_set_tuning("nodecls_t", v)
int& nodecls_t_flag() {
    static int on = [] {
        const char* e = getenv("FPM_NODECLS_T");
        return e ? atoi(e) : 1;
    }();
    return on;
}

// MLP on packed fp32 FMAs (default) or scalar FMAs (bit-identical); env FPM_GNN_PACKED or
// fpm_set_tuning("gnn_packed", v)
int& gnn_packed_flag() {
    static int on = [] {
        const char* e = getenv("FPM_GNN_PACKED");
        return e ? atoi(e) : 1;
    }();
    return on;
}

// graph-2 nodes per workgroup, processed by parallel 256-thread groups (1, 2, 4; bit-identical);
// env FPM_GNN_GROUP or fpm_set_tuning("gnn_group", v)
int& gnn_group_flag() {
    static int u = [] {
        const char* e = getenv("FPM_GNN_GROUP");
        return e ? atoi(e) : 2;
    }();
    return u;
}

// the grouping for the first (1-channel) layer as well: env FPM_GNN_GROUP1 / "gnn_group1"
int& gnn_group1_flag() {
    static int u = [] {
        const char* e = getenv("FPM_GNN_GROUP1");
        return e ? atoi(e) : 0;
    }();
    return u;
}

// 16-B phase-1 loads for the 17-channel layer (bit-identical); env FPM_GNN_WIDE or
// fpm_set_tuning("gnn_wide", v)
int& gnn_wide_flag() {
    static int u = [] {
        const char* e = getenv("FPM_GNN_WIDE");
        return e ? atoi(e) : 0;
    }();
    return u;
}

// input-channel-outer MLP order (wide scalar weight loads, bit-identical); env FPM_GNN_IL or
// fpm_set_tuning("gnn_il", v)
int& gnn_il_flag() {
    static int u = [] {
        const char* e = getenv("FPM_GNN_IL");
        return e ? atoi(e) : 0;
    }();
    return u;
}

// graph-2 neighbour rows loaded U at a time (1, 2 or 3; bit-identical); env FPM_GNN_UNROLL or
// fpm_set_tuning("gnn_unroll", v)
int& gnn_unroll_flag() {
    static int u = [] {
        const char* e = getenv("FPM_GNN_UNROLL");
        return e ? atoi(e) : 1;
    }();
    return u;
}

extern "C" int fpm_kron_gnn_layer_fwd(const float* X, int C, int B, int n1max, int n2max, const int* ptr1,
                                      const int* nbr1, const int* ptr2, const int* nbr2, const int* n1, const int* n2,
                                      const float* params, float* Xout, float* zbuf, float* vpart, const float* cls_w,
                                      void* stream) {
    FPM_CHECK_ARG(C == 1 || C == 17, "gnn_layer: C must be 1 or 17 (got %d)", C);
    FPM_CHECK_ARG(!vpart || cls_w, "gnn_layer: vpart needs cls_w");
    if (B == 0) return 0;
    FPM_CHECK_ARG(n1max <= 1024, "gnn_layer: n1max must be <= 1024");
    FPM_CHECK_ARG((long)C * n1max * n2max * 4 < (1L << 31), "gnn_layer: a pair's state must be < 2 GiB");
    dim3 grid(pair_grid(n2max, B));
    hipStream_t st = (hipStream_t)stream;
    const size_t sh = (size_t)(C == 1 ? 1 : 20) * n1max * 4;
    const int threads = (n1max + 63) / 64 * 64;
    const bool packed = gnn_packed_flag() != 0;
    const int un = gnn_unroll_flag();
    // default 2 (21% faster at n = 256, 13% at n = 100; slower as a 1024-thread workgroup at n = 512)
    const int grp = gnn_group_flag() * threads <= 512 ? gnn_group_flag() : 1;
    const bool wide = gnn_wide_flag() != 0 && (n1max & 3) == 0;
    const bool il = gnn_il_flag() != 0;
#define FPM_GNN_WI(C_, P_, U_, G_, W_, I_)                                                                       \
    do {                                                                                                         \
        const size_t sh_ = sh * G_;                                                                              \
        if (sh_ > 65536)                                                                                         \
            (void)hipFuncSetAttribute((const void*)gnn_layer_kernel<C_, P_, U_, G_, W_, I_>,                     \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh_);                     \
        const dim3 g_(pair_grid((n2max + G_ - 1) / G_, B));                                                      \
        const dim3 t_(threads * G_);                                                                             \
        hipLaunchKernelGGL((gnn_layer_kernel<C_, P_, U_, G_, W_, I_>), g_, t_, sh_, st, X, n1max, n2max, ptr1,   \
                           nbr1, ptr2, nbr2, n1, n2, params, Xout, zbuf, vpart, cls_w, B);                       \
    } while (0)
#define FPM_GNN_W(C_, P_, U_, G_, W_)                                                                            \
    do {                                                                                                         \
        if (il) FPM_GNN_WI(C_, P_, U_, G_, W_, true);                                                            \
        else FPM_GNN_WI(C_, P_, U_, G_, W_, false);                                                              \
    } while (0)
#define FPM_GNN(C_, P_, U_, G_) FPM_GNN_W(C_, P_, U_, G_, false)
    if (C == 1) {
        if (!packed) FPM_GNN(1, false, 1, 1);
        else if (grp == 2 && gnn_group1_flag()) FPM_GNN(1, true, 1, 2);
        else FPM_GNN(1, true, 1, 1);
    }
    else if (!packed) FPM_GNN(17, false, 1, 1);
    else if (wide && grp == 2) FPM_GNN_W(17, true, 1, 2, true);
    else if (wide) FPM_GNN_W(17, true, 1, 1, true);
    else if (grp == 2) FPM_GNN(17, true, 1, 2);
    else if (grp == 4) FPM_GNN(17, true, 1, 4);
    else if (un == 2) FPM_GNN(17, true, 2, 1);
    else if (un == 3) FPM_GNN(17, true, 3, 1);
    else FPM_GNN(17, true, 1, 1);
#undef FPM_GNN
#undef FPM_GNN_W
#undef FPM_GNN_WI
    return fpm::check_launch("fpm_kron_gnn_layer_fwd");
}

extern "C" int fpm_gnn_param_count(int C) { return C == 1 ? GnnPack<1>::total : GnnPack<17>::total; }

extern "C" int fpm_node_classifier(const float* X, int B, int n1max, int n2max, const float* w, const float* bias,
                                   const float* vpart, float* s, void* stream) {
    if (B == 0) return 0;
    if (nodecls_t_flag() && B <= 65535) {
        const dim3 grid((unsigned)((n1max + 63) / 64), (unsigned)((n2max + 63) / 64), (unsigned)B);
        hipLaunchKernelGGL(node_classifier_t_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, n1max, n2max, w, bias,
                           vpart, s);
        return fpm::check_launch("fpm_node_classifier");
    }
    hipLaunchKernelGGL(node_classifier_kernel, dim3(pair_grid(n2max, B)), dim3(256), 0, (hipStream_t)stream, X, n1max,
                       n2max, w, bias, vpart, s, B);
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
                                                        int adj, float* __restrict__ out, int B) {
    extern __shared__ float T[];
    int d, b;
    if (!pair_block(n2max, B, b, d)) return;
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
        out[(long)b * C * N + (long)c * N + (long)d * n1max + i] = adj ? acc : (dn > 0.f ? acc / dn : 0.f);
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
                                                          int adj, float* __restrict__ out, int B) {
    extern __shared__ float T[];                           // [i][C] node-major
    int d, b;
    if (!pair_block(n2max, B, b, d)) return;
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
        const float r = adj ? a : a * rdn;
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
