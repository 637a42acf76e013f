// On-device keypoint-graph construction: replaces the DataLoader-side
// utils/build_graphs.py:12-120 ('tri' / 'fc' / 'near', sym=True), GMDataset.to_pyg_graph's edge
// list + pseudo-coordinates (src/gmdataset.py:170-189) and the collate's Kronecker index lists
// (src/gmdataset.py:614-642: CSCMatrix3d(kron(G2, G1)).indices, CSCMatrix3d(kron(H2, H1)).T.indices).
//
// Delaunay ('tri') without a triangulation: an edge (i, j) belongs to the Delaunay graph iff some
// circle through p_i and p_j has no point strictly inside.  The centres of those circles lie on
// the bisector c(t) = m + t.nrm (m = midpoint, nrm = (p_j - p_i) rotated by 90 degrees); point k
// with side s_k = nrm.(p_k - m) and num_k = |m - p_i|^2 - |m - p_k|^2 is inside circle(t) iff
// t > num_k/(-2 s_k) for s_k > 0, iff t < num_k/(-2 s_k) for s_k < 0.  So the edge exists iff
//     max_{s_k<0} num_k/|s_k|  <  min_{s_k>0} -num_k/s_k
// (strict: four cocircular points leave both diagonals out; Qhull's 'Qt' would pick one), and a
// point strictly inside the segment (s_k = 0, num_k > 0) kills it.  Hull edges have one side empty.
// Each lane owns one candidate pair (i < j) and streams k through LDS, comparing the fractions by
// cross-multiplication in fp64 (the orientation s_k of fp32 inputs is exact in fp64); a pair stops
// as soon as max >= min.  Non-edges die after a few dozen points, so a lane pulls the next pair
// from a block-wide LDS counter (persistent lanes, no divergence between the pair streams) and
// only the ~3n true edges run the full n-point pass.  Result: a symmetric adjacency bit matrix.
// Degenerate inputs as build_graphs.py:89-100: n < 3 and all-collinear point sets (QhullError)
// give the fully connected graph.  General position is assumed otherwise (no duplicate points,
// no four cocircular points): there the Delaunay graph is unique and equals scipy's.
#include "fpm_common.h"

namespace {

constexpr int GB_THREADS = 256;
constexpr int GB_UNROLL = 4;
constexpr int GB_MAX_N = 1024;

__device__ __forceinline__ unsigned lane_rank(unsigned long long mask) {
    const unsigned lo = __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u);
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), lo);
}

// strictly-upper pair index p -> (i, j), i < j < n; row i starts at i*(2n-1-i)/2
__device__ __forceinline__ void tri_decode(long p, int n, int& i, int& j) {
    const double b = 2.0 * n - 1.0;
    int r = (int)((b - sqrt(b * b - 8.0 * (double)p)) * 0.5);
    r = r < 0 ? 0 : (r > n - 2 ? n - 2 : r);
    while (r > 0 && (long)r * (2 * n - 1 - r) / 2 > p) --r;
    while (r < n - 2 && (long)(r + 1) * (2 * n - 2 - r) / 2 <= p) ++r;
    i = r;
    j = (int)(p - (long)r * (2 * n - 1 - r) / 2) + r + 1;
}

struct PairTest {
    double mx, my, nx, ny, r2;
    double aL, bL, aR, bR;  // max_{s<0} aL/bL, min_{s>0} aR/bR (denominators > 0)
    int i, j, k;
    bool hasL, hasR, dead;

    __device__ __forceinline__ void init(const double2* pts, int pi, int pj) {
        const double2 a = pts[pi], b = pts[pj];
        i = pi;
        j = pj;
        mx = (a.x + b.x) * 0.5;
        my = (a.y + b.y) * 0.5;
        const double dx = b.x - a.x, dy = b.y - a.y;
        nx = -dy;
        ny = dx;
        r2 = 0.25 * (dx * dx + dy * dy);
        aL = bL = aR = bR = 0.0;
        hasL = hasR = false;
        dead = (dx == 0.0 && dy == 0.0);  // duplicate points: no edge
        k = 0;
    }

    __device__ __forceinline__ void step(const double2* pts, int kk) {
        if (kk == i || kk == j) return;
        const double2 c = pts[kk];
        const double ux = c.x - mx, uy = c.y - my;
        const double s = nx * ux + ny * uy;
        const double num = r2 - (ux * ux + uy * uy);
        if (s < 0.0) {
            const double bs = -s;
            if (!hasL || num * bL > aL * bs) {
                aL = num;
                bL = bs;
                hasL = true;
            }
        } else if (s > 0.0) {
            const double an = -num;
            if (!hasR || an * bR < aR * s) {
                aR = an;
                bR = s;
                hasR = true;
            }
        } else if (num > 0.0) {
            dead = true;  // collinear point strictly between p_i and p_j
        }
    }

    __device__ __forceinline__ void check() {
        if (hasL && hasR && aL * bR >= aR * bL) dead = true;
    }
};

// one block per graph: adjacency bits (G, nmax, W) u32, row degrees (G, nmax), edge count (G),
// optional dense A (G, nmax, nmax) fp32 (build_graphs' A)
__global__ __launch_bounds__(GB_THREADS) void graph_adj_kernel(const float* __restrict__ P, const int* __restrict__ nv,
                                                               int nmax, int W, int strat, double thre,
                                                               uint32_t* __restrict__ adj, int* __restrict__ deg,
                                                               int* __restrict__ ecount, float* __restrict__ Adense) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double2* pts = (double2*)smem;
    uint32_t* bits = (uint32_t*)(pts + nmax);
    __shared__ unsigned long long s_next;
    __shared__ int s_ref, s_nondeg, s_cnt;
    const int g = blockIdx.x, tid = threadIdx.x;
    const int n = min(nv[g], nmax);
    const float* Pg = P + (long)g * nmax * 2;
    for (int t = tid; t < nmax; t += GB_THREADS)
        pts[t] = t < n ? make_double2((double)Pg[2 * t], (double)Pg[2 * t + 1]) : make_double2(0.0, 0.0);
    for (int t = tid; t < nmax * W; t += GB_THREADS) bits[t] = 0u;
    if (tid == 0) {
        s_next = 0ull;
        s_ref = n;
        s_nondeg = 0;
        s_cnt = 0;
    }
    __syncthreads();

    int mode = strat;  // 0 tri, 1 fc, 2 near
    if (mode == 0 && n < 3) mode = 1;  // build_graphs.py:89-90
    if (mode == 0) {
        // Qhull rejects an all-collinear (flat) input -> fully connected (build_graphs.py:96-100)
        const double2 p0 = pts[0];
        for (int t = tid + 1; t < n; t += GB_THREADS)
            if (pts[t].x != p0.x || pts[t].y != p0.y) atomicMin(&s_ref, t);
        __syncthreads();
        const int a = s_ref;
        if (a < n) {
            const double ax = pts[a].x - p0.x, ay = pts[a].y - p0.y;
            for (int t = tid; t < n; t += GB_THREADS) {
                const double cr = ax * (pts[t].y - p0.y) - ay * (pts[t].x - p0.x);
                if (cr != 0.0) s_nondeg = 1;
            }
        }
        __syncthreads();
        if (!s_nondeg) mode = 1;
    }

    if (mode != 0) {
        for (int t = tid; t < n * W; t += GB_THREADS) {
            const int i = t / W, w = t - i * W;
            uint32_t m = 0u;
            for (int b = 0; b < 32; ++b) {
                const int j = w * 32 + b;
                if (j >= n || j == i) continue;
                bool keep = true;
                if (mode == 2) {
                    const double dx = pts[i].x - pts[j].x, dy = pts[i].y - pts[j].y;
                    keep = !(sqrt(dx * dx + dy * dy) > thre);
                }
                if (keep) m |= 1u << b;
            }
            bits[t] = m;
        }
    } else {
        const long npairs = (long)n * (n - 1) / 2;
        const int lane = tid & (FPM_WAVE - 1);
        PairTest st;
        bool active = false;
        // first 64 pairs of this wave
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(&s_next, (unsigned long long)FPM_WAVE);
        base = __shfl(base, 0);
        {
            const long p = (long)base + lane;
            active = p < npairs;
            if (active) {
                int i, j;
                tri_decode(p, n, i, j);
                st.init(pts, i, j);
            }
        }
        while (true) {
            if (active) {
#pragma unroll
                for (int u = 0; u < GB_UNROLL; ++u) st.step(pts, min(st.k + u, n - 1));
                st.k += GB_UNROLL;
                st.check();
            }
            const bool done = active && (st.dead || st.k >= n);
            if (done && !st.dead) {
                atomicOr(&bits[st.i * W + (st.j >> 5)], 1u << (st.j & 31));
                atomicOr(&bits[st.j * W + (st.i >> 5)], 1u << (st.i & 31));
            }
            const unsigned long long dm = __ballot(done);
            if (dm) {
                unsigned long long b2 = 0;
                if (lane == 0) b2 = atomicAdd(&s_next, (unsigned long long)__popcll(dm));
                b2 = __shfl(b2, 0);
                if (done) {
                    const long p = (long)b2 + lane_rank(dm);
                    active = p < npairs;
                    if (active) {
                        int i, j;
                        tri_decode(p, n, i, j);
                        st.init(pts, i, j);
                    }
                }
            }
            if (!__ballot(active)) break;
        }
    }
    __syncthreads();

    uint32_t* ag = adj + (long)g * nmax * W;
    for (int t = tid; t < nmax * W; t += GB_THREADS) ag[t] = bits[t];
    int local = 0;
    for (int i = tid; i < nmax; i += GB_THREADS) {
        int d = 0;
        for (int w = 0; w < W; ++w) d += __popc(bits[i * W + w]);
        deg[(long)g * nmax + i] = d;
        local += d;
    }
    atomicAdd(&s_cnt, local);
    if (Adense) {
        float* Ag = Adense + (long)g * nmax * nmax;
        for (long t = tid; t < (long)nmax * nmax; t += GB_THREADS) {
            const int i = (int)(t / nmax), j = (int)(t - (long)i * nmax);
            Ag[t] = (bits[i * W + (j >> 5)] >> (j & 31)) & 1u ? 1.f : 0.f;
        }
    }
    __syncthreads();
    if (tid == 0) ecount[g] = s_cnt;
}

// one block per graph: edge list in np.nonzero(A) row-major order with batch-global node ids
// (graph g's node i -> g*nmax + i), pseudo = clip(0.5*(P_src - P_dst)/rescale + 0.5, 0, 1) in fp64
// rounded to fp32 (gmdataset.py:172-176), edge offsets, optional incidence G/H (build_graphs.py:64-74).
__global__ __launch_bounds__(GB_THREADS) void graph_edges_kernel(
    const float* __restrict__ P, const uint32_t* __restrict__ adj, const int* __restrict__ deg,
    const int* __restrict__ ecount, int G, int nmax, int W, double rescale, int* __restrict__ src,
    int* __restrict__ dst, float* __restrict__ pseudo, long* __restrict__ edge_off, float* __restrict__ Ginc,
    float* __restrict__ Hinc, int epad) {
    __shared__ long s_red[GB_THREADS / FPM_WAVE];
    __shared__ int s_rowoff[GB_MAX_N];
    __shared__ int s_wsum[GB_THREADS / FPM_WAVE];
    const int g = blockIdx.x, tid = threadIdx.x;
    const int lane = tid & (FPM_WAVE - 1), wv = tid / FPM_WAVE;
    long part = 0;
    for (int t = tid; t < g; t += GB_THREADS) part += ecount[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    if (lane == 0) s_red[wv] = part;
    // exclusive scan of row degrees: thread-contiguous chunks of R rows
    const int R = (nmax + GB_THREADS - 1) / GB_THREADS;
    const int* dg = deg + (long)g * nmax;
    int run = 0;
    for (int r = 0; r < R; ++r) {
        const int i = tid * R + r;
        if (i < nmax) {
            s_rowoff[i] = run;
            run += dg[i];
        }
    }
    int incl = run;
#pragma unroll
    for (int o = 1; o < FPM_WAVE; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == FPM_WAVE - 1) s_wsum[wv] = incl;
    __syncthreads();
    long goff = 0;
    for (int w = 0; w < GB_THREADS / FPM_WAVE; ++w) goff += s_red[w];
    int woff = 0;
    for (int w = 0; w < wv; ++w) woff += s_wsum[w];
    const int texcl = woff + incl - run;
    for (int r = 0; r < R; ++r) {
        const int i = tid * R + r;
        if (i < nmax) s_rowoff[i] += texcl;
    }
    __syncthreads();
    if (edge_off) {
        if (tid == 0) edge_off[g] = goff;
        if (tid == 0 && g == G - 1) edge_off[G] = goff + ecount[g];
    }
    const float* Pg = P + (long)g * nmax * 2;
    const uint32_t* ag = adj + (long)g * nmax * W;
    for (int i = tid; i < nmax; i += GB_THREADS) {
        int el = s_rowoff[i];
        const double pix = (double)Pg[2 * i], piy = (double)Pg[2 * i + 1];
        for (int w = 0; w < W; ++w) {
            uint32_t m = ag[i * W + w];
            while (m) {
                const int b = __builtin_ctz(m);
                m &= m - 1u;
                const int j = w * 32 + b;
                const long e = goff + el;
                src[e] = g * nmax + i;
                dst[e] = g * nmax + j;
                double qx = 0.5 * (pix - (double)Pg[2 * j]) / rescale + 0.5;
                double qy = 0.5 * (piy - (double)Pg[2 * j + 1]) / rescale + 0.5;
                qx = qx < 0.0 ? 0.0 : (qx > 1.0 ? 1.0 : qx);
                qy = qy < 0.0 ? 0.0 : (qy > 1.0 ? 1.0 : qy);
                pseudo[2 * e] = (float)qx;
                pseudo[2 * e + 1] = (float)qy;
                if (Ginc && el < epad) {
                    Ginc[((long)g * nmax + i) * epad + el] = 1.f;
                    Hinc[((long)g * nmax + j) * epad + el] = 1.f;
                }
                ++el;
            }
        }
    }
}

// Kronecker index lists of one pair (collate, gmdataset.py:623-634): for edge pair
// c = e2*E1 + e1 (kron(G2, G1) column order) rowG[c] = src2[e2]*n1pad + src1[e1] (the CSC row
// index of the single nonzero of column c) and colH[c] = dst2[e2]*n1pad + dst1[e1] (the
// transposed kron(H2, H1)); written as float32 like the reference's `.float()` use (ngm.py:339),
// or int64.  Edge ids are local (node ids relative to the graph).
template <typename T>
__global__ void kron_pattern_kernel(const int* __restrict__ src1, const int* __restrict__ dst1, long E1,
                                    const int* __restrict__ src2, const int* __restrict__ dst2, long E2,
                                    int base1, int base2, int n1pad, T* __restrict__ rowG, T* __restrict__ colH) {
    const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= E1 * E2) return;
    const long e2 = c / E1, e1 = c - e2 * E1;
    const long r = (long)(src2[e2] - base2) * n1pad + (src1[e1] - base1);
    const long q = (long)(dst2[e2] - base2) * n1pad + (dst1[e1] - base1);
    rowG[c] = (T)r;
    colH[c] = (T)q;
}

}  // namespace

extern "C" int fpm_graph_words(int nmax) { return (nmax + 31) / 32; }

extern "C" int fpm_graph_build(const float* P, const int* n, int G, int nmax, int strategy, double thre,
                               uint32_t* adj, int* deg, int* ecount, float* Adense, void* stream) {
    FPM_CHECK_ARG(G >= 0 && nmax >= 0 && nmax <= GB_MAX_N, "graph_build: need 0 <= nmax <= %d (got %d)",
                  GB_MAX_N, nmax);
    FPM_CHECK_ARG(strategy >= 0 && strategy <= 2, "graph_build: strategy must be 0 (tri), 1 (fc) or 2 (near)");
    if (G == 0 || nmax == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int W = fpm_graph_words(nmax);
    const size_t sh = (size_t)nmax * sizeof(double2) + (size_t)nmax * W * sizeof(uint32_t);
    if (sh > 65536) {
        const hipError_t e = hipFuncSetAttribute((const void*)graph_adj_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        FPM_CHECK_ARG(e == hipSuccess, "graph_build: %zu B of LDS refused: %s", sh, hipGetErrorString(e));
    }
    hipLaunchKernelGGL(graph_adj_kernel, dim3(G), dim3(GB_THREADS), sh, st, P, n, nmax, W, strategy, thre, adj, deg,
                       ecount, Adense);
    return fpm::check_launch("fpm_graph_build");
}

extern "C" int fpm_graph_edges(const float* P, const uint32_t* adj, const int* deg, const int* ecount, int G, int nmax,
                               double rescale, int* src, int* dst, float* pseudo, long* edge_off, float* Ginc,
                               float* Hinc, int epad, void* stream) {
    FPM_CHECK_ARG(G >= 0 && nmax >= 0 && nmax <= GB_MAX_N, "graph_edges: need 0 <= nmax <= %d", GB_MAX_N);
    FPM_CHECK_ARG((Ginc == nullptr) == (Hinc == nullptr), "graph_edges: pass both G and H incidence or neither");
    if (G == 0 || nmax == 0) return 0;
    hipLaunchKernelGGL(graph_edges_kernel, dim3(G), dim3(GB_THREADS), 0, (hipStream_t)stream, P, adj, deg, ecount, G,
                       nmax, fpm_graph_words(nmax), rescale, src, dst, pseudo, edge_off, Ginc, Hinc, epad);
    return fpm::check_launch("fpm_graph_edges");
}

// out_dtype: 0 = float32, 1 = int64
extern "C" int fpm_kron_pattern(const int* src1, const int* dst1, long E1, const int* src2, const int* dst2, long E2,
                                int base1, int base2, int n1pad, int out_dtype, void* rowG, void* colH, void* stream) {
    FPM_CHECK_ARG(E1 >= 0 && E2 >= 0 && n1pad > 0, "kron_pattern: bad sizes");
    FPM_CHECK_ARG(out_dtype == 0 || out_dtype == 1, "kron_pattern: out_dtype must be 0 (f32) or 1 (i64)");
    const long tot = E1 * E2;
    if (tot == 0) return 0;
    const dim3 grid((unsigned)((tot + 255) / 256));
    if (out_dtype == 0)
        hipLaunchKernelGGL(kron_pattern_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, src1, dst1, E1, src2,
                           dst2, E2, base1, base2, n1pad, (float*)rowG, (float*)colH);
    else
        hipLaunchKernelGGL(kron_pattern_kernel<long>, grid, dim3(256), 0, (hipStream_t)stream, src1, dst1, E1, src2,
                           dst2, E2, base1, base2, n1pad, (long*)rowG, (long*)colH);
    return fpm::check_launch("fpm_kron_pattern");
}
