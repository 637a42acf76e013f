// SplineConv message passing (PyG 1.6.3 SplineConv(768, 768, dim=2, kernel_size=5, aggr='max')
// as used by the reference's SConv, src/model/spline_conv.py:17,28-41, and the Siamese
// residual x + 0.1*SConv(x), spline_conv.py:51-57).
//
// MI355X design: edges of the whole side-batch are bucketed by their B-spline group
// g = (floor(4u0), floor(4u1)) (25 groups; every edge of group g uses the same 4 kernel cells), so
// a layer is one grouped MFMA GEMM with K = 4 x 768 (A = gathered source rows, B = the 4 cells'
// [out][in] weights, fp32 basis applied per segment) writing one message row per edge, plus the
// root GEMM x R, plus a segmented max over each node's in-edges fused with root/bias/ReLU or the
// residual.  The bucketing plan (basis, group offsets, tile table, dst CSR) is built on device
// once per side and shared by both layers.
#include "gemm_core.h"

#include <vector>

namespace {

// optional HIP-event timing of the dominant kernel (edge-message GEMM), read by bench.py
struct ProfRec {
    hipEvent_t a, b;
    double flops;
};
bool g_prof_on = false;
std::vector<ProfRec> g_prof;



struct PlanLayout {
    long cnt, grp_off, slot, dslot, gidx, indeg, dst_ptr, rows_src, rows_basis, dst_rows, nbr_local, tile_info,
        total;
};

__host__ __device__ inline long al(long x) { return (x + 255) & ~255L; }

PlanLayout plan_layout(long E, long num_nodes, long max_tiles) {
    PlanLayout L;
    long o = 0;
    L.cnt = o; o += al(32 * 4);
    L.grp_off = o; o += al(32 * 4);
    L.slot = o; o += al(E * 4);
    L.dslot = o; o += al(E * 4);
    L.gidx = o; o += al(E * 4);
    L.indeg = o; o += al(num_nodes * 4);
    L.dst_ptr = o; o += al((num_nodes + 1) * 4);
    L.rows_src = o; o += al(E * 4);
    L.rows_basis = o; o += al(E * 16);
    L.dst_rows = o; o += al(E * 4);
    L.nbr_local = o; o += al(E * 4);
    L.tile_info = o; o += al(max_tiles * 8);
    L.total = o;
    return L;
}

// per-edge basis + group; slots within a group come from a block-local LDS histogram plus one
// global atomic per (block, group) (25 global counters would otherwise serialise 1.5M atomics)
__global__ __launch_bounds__(256) void plan_count_kernel(const int* __restrict__ src, const int* __restrict__ dst,
                                                         const float* __restrict__ pseudo, long E, int* cnt, int* slot,
                                                         int* dslot, int* gidx, int* indeg, float* basis_tmp) {
    __shared__ int lcnt[32], lbase[32];
    if (threadIdx.x < 32) lcnt[threadIdx.x] = 0;
    __syncthreads();
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    int g = -1, lslot = 0;
    if (e < E) {
        // torch-spline-conv basis, open spline degree 1: v = u * (kernel - 1), frac, floor
        int f[2];
        float fr[2];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            float v = pseudo[2 * e + d] * 4.0f;
            float fl = floorf(v);
            f[d] = (int)fl;
            fr[d] = v - fl;
        }
        float b4[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            float b = 1.0f;
            b = b * ((s & 1) ? fr[0] : 1.0f - fr[0]);
            b = b * ((s >> 1) ? fr[1] : 1.0f - fr[1]);
            b4[s] = b;
        }
        g = f[0] + 5 * f[1];
        gidx[e] = g;
        lslot = atomicAdd(&lcnt[g], 1);
        dslot[e] = atomicAdd(&indeg[dst[e]], 1);
        *(float4*)(basis_tmp + 4 * e) = make_float4(b4[0], b4[1], b4[2], b4[3]);
    }
    __syncthreads();
    if (threadIdx.x < 25) {
        int c = lcnt[threadIdx.x];
        lbase[threadIdx.x] = c ? atomicAdd(&cnt[threadIdx.x], c) : 0;
    }
    __syncthreads();
    if (e < E) slot[e] = lbase[g] + lslot;
}

__global__ __launch_bounds__(1024) void plan_scan_kernel(const int* cnt, int* grp_off, int* tile_info,
                                                         int max_tiles, const int* indeg, int* dst_ptr,
                                                         long num_nodes) {
    __shared__ int part[1024];
    __shared__ int tilebuf[16384];
    __shared__ int ntile_total;
    const int tid = threadIdx.x;
    if (tid == 0) {
        int off = 0, t = 0;
        for (int g = 0; g < 25; ++g) {
            grp_off[g] = off;
            int c = cnt[g];
            for (int r = 0; r < c; r += fpm::GBM) {
                tile_info[2 * t] = g;
                tile_info[2 * t + 1] = off + r;
                ++t;
            }
            off += c;
        }
        grp_off[25] = off;
        ntile_total = t;
    }
    __syncthreads();
    for (int t = ntile_total + tid; t < max_tiles; t += 1024) {
        tile_info[2 * t] = -1;
        tile_info[2 * t + 1] = 0;
    }
    // exclusive scan of indeg -> dst_ptr, tiled through LDS (coalesced global reads/writes)
    constexpr int TILE = 16384, PER = TILE / 1024;
    int* buf = tilebuf;
    int carry = 0;
    for (long t0 = 0; t0 < num_nodes; t0 += TILE) {
        const int len = (int)(num_nodes - t0 < TILE ? num_nodes - t0 : TILE);
        for (int k = tid; k < TILE; k += 1024) buf[k] = k < len ? indeg[t0 + k] : 0;
        __syncthreads();
        int loc[PER];
        int s = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            loc[k] = s;
            s += buf[tid * PER + k];
        }
        part[tid] = s;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            int v = tid >= o ? part[tid - o] : 0;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        const int base = carry + part[tid] - s;
#pragma unroll
        for (int k = 0; k < PER; ++k) buf[tid * PER + k] = base + loc[k];
        const int total = part[1023];
        __syncthreads();
        for (int k = tid; k < len; k += 1024) dst_ptr[t0 + k] = buf[k];
        carry += total;
        __syncthreads();
    }
    if (tid == 0) dst_ptr[num_nodes] = carry;
}

__global__ void plan_fill_kernel(const int* __restrict__ src, const int* __restrict__ dst, long E, int nmax,
                                 const int* __restrict__ grp_off, const int* __restrict__ slot,
                                 const int* __restrict__ dslot, const int* __restrict__ gidx,
                                 const int* __restrict__ dst_ptr, const float* __restrict__ basis_tmp, int* rows_src,
                                 float* rows_basis, int* dst_rows, int* nbr_local) {
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    int row = grp_off[gidx[e]] + slot[e];
    int s = src[e], d = dst[e];
    rows_src[row] = s;
    *(float4*)(rows_basis + 4 * (long)row) = *(const float4*)(basis_tmp + 4 * e);
    int p = dst_ptr[d] + dslot[e];
    dst_rows[p] = row;
    nbr_local[p] = s % nmax;
}

// Deterministic in-edge order per node (ascending source): the atomics above fill each list in
// arbitrary order, and the GNN aggregation sums over these lists in fp32.
__global__ void plan_sort_kernel(const int* __restrict__ dst_ptr, long num_nodes, int* __restrict__ dst_rows,
                                 int* __restrict__ nbr_local) {
    long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= num_nodes) return;
    const int beg = dst_ptr[v], end = dst_ptr[v + 1];
    for (int a = beg + 1; a < end; ++a) {
        int kn = nbr_local[a], kr = dst_rows[a];
        int b = a - 1;
        while (b >= beg && nbr_local[b] > kn) {
            nbr_local[b + 1] = nbr_local[b];
            dst_rows[b + 1] = dst_rows[b];
            --b;
        }
        nbr_local[b + 1] = kn;
        dst_rows[b + 1] = kr;
    }
}

// out[v] = max_{in-edges} msg + root[v] + bias  -> RELU: relu(.) ; RESID: x[v] + 0.1 * (.)
template <typename T>
__global__ __launch_bounds__(256) void segmax_kernel(const T* __restrict__ msg, const float* __restrict__ root,
                                                     const float* __restrict__ bias, const int* __restrict__ dst_ptr,
                                                     const int* __restrict__ dst_rows, long num_nodes, int nmax,
                                                     const int* __restrict__ nvalid, int mode,
                                                     const float* __restrict__ xres, const float* __restrict__ cscale,
                                                     float* __restrict__ out_f, T* __restrict__ out_t) {
    const int lane = threadIdx.x & 63;
    long v = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= num_nodes) return;
    const int b = (int)(v / nmax), loc = (int)(v - (long)b * nmax);
    const bool valid = loc < nvalid[b];
    const int beg = dst_ptr[v], end = dst_ptr[v + 1];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        const int c0 = 4 * lane + 256 * t;
        float m[4];
        if (beg < end) {
            m[0] = m[1] = m[2] = m[3] = -INFINITY;
            for (int e = beg; e < end; ++e) {
                const T* row = msg + (long)dst_rows[e] * 768 + c0;
#pragma unroll
                for (int j = 0; j < 4; ++j) m[j] = fmaxf(m[j], fpm::to_f<T>(row[j]));
            }
        } else {
            m[0] = m[1] = m[2] = m[3] = 0.f;   // torch_scatter max: empty segment -> 0
        }
        float y[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float o = (m[j] + root[v * 768 + c0 + j]) + bias[c0 + j];
            if (mode == 0) y[j] = fmaxf(o, 0.f);
            else y[j] = xres[v * 768 + c0 + j] + 0.1f * o;
            if (!valid) y[j] = 0.f;
        }
        if (out_f) {
#pragma unroll
            for (int j = 0; j < 4; ++j) out_f[v * 768 + c0 + j] = y[j];
        }
        if (out_t) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float z = cscale ? y[j] * cscale[(long)b * 768 + c0 + j] : y[j];
                out_t[v * 768 + c0 + j] = fpm::from_f<T>(z);
            }
        }
    }
}

}  // namespace

extern "C" long fpm_spline_plan_bytes(long E, long num_nodes) {
    long max_tiles = (E + fpm::GBM - 1) / fpm::GBM + 25;
    return plan_layout(E, num_nodes, max_tiles).total + al(E * 16);
}

extern "C" int fpm_spline_plan(const int* src, const int* dst, const float* pseudo, long E, long num_nodes, int nmax,
                               void* ws, long ws_bytes, void* stream) {
    long max_tiles = (E + fpm::GBM - 1) / fpm::GBM + 25;
    PlanLayout L = plan_layout(E, num_nodes, max_tiles);
    FPM_CHECK_ARG(ws_bytes >= fpm_spline_plan_bytes(E, num_nodes), "spline_plan: workspace too small");
    FPM_CHECK_ARG(E > 0 && num_nodes > 0 && nmax > 0, "spline_plan: bad sizes");
    char* w = (char*)ws;
    hipStream_t st = (hipStream_t)stream;
    float* basis_tmp = (float*)(w + L.total);
    (void)hipMemsetAsync(w + L.cnt, 0, 32 * 4, st);
    (void)hipMemsetAsync(w + L.indeg, 0, num_nodes * 4, st);
    int blocks = (int)((E + 255) / 256);
    hipLaunchKernelGGL(plan_count_kernel, dim3(blocks), dim3(256), 0, st, src, dst, pseudo, E, (int*)(w + L.cnt),
                       (int*)(w + L.slot), (int*)(w + L.dslot), (int*)(w + L.gidx), (int*)(w + L.indeg), basis_tmp);
    hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(1024), 0, st, (const int*)(w + L.cnt), (int*)(w + L.grp_off),
                       (int*)(w + L.tile_info), (int)max_tiles, (const int*)(w + L.indeg), (int*)(w + L.dst_ptr),
                       num_nodes);
    hipLaunchKernelGGL(plan_fill_kernel, dim3(blocks), dim3(256), 0, st, src, dst, E, nmax, (const int*)(w + L.grp_off),
                       (const int*)(w + L.slot), (const int*)(w + L.dslot), (const int*)(w + L.gidx),
                       (const int*)(w + L.dst_ptr), (const float*)basis_tmp, (int*)(w + L.rows_src),
                       (float*)(w + L.rows_basis), (int*)(w + L.dst_rows), (int*)(w + L.nbr_local));
    hipLaunchKernelGGL(plan_sort_kernel, dim3((unsigned)((num_nodes + 255) / 256)), dim3(256), 0, st,
                       (const int*)(w + L.dst_ptr), num_nodes, (int*)(w + L.dst_rows), (int*)(w + L.nbr_local));
    return fpm::check_launch("fpm_spline_plan");
}

// Pointers into the plan for the GNN layer (dst CSR with local neighbour indices).
extern "C" int fpm_spline_plan_csr(void* ws, long E, long num_nodes, int** dst_ptr, int** nbr_local) {
    long max_tiles = (E + fpm::GBM - 1) / fpm::GBM + 25;
    PlanLayout L = plan_layout(E, num_nodes, max_tiles);
    *dst_ptr = (int*)((char*)ws + L.dst_ptr);
    *nbr_local = (int*)((char*)ws + L.nbr_local);
    return 0;
}

// One SplineConv layer over a whole side-batch.
//   mode 0: out = relu(max_e msg + x R + b)            (conv 0 + F.relu, spline_conv.py:35)
//   mode 1: out = xres + 0.1 * (max_e msg + x R + b)   (conv 1 + Siamese residual, :38, :56)
// x_op: operand copy of the input (dtype); W: (25, 768 out, 768 in); R: (768 out, 768 in).
// msg_ws: (E, 768) dtype; root_ws: (num_nodes, 768) f32.  cscale (B,768) optionally scales the
// operand output (X o c for the vertex affinity, affinity_layer.py:15).
extern "C" int fpm_spline_conv_fwd(int dtype, const void* x_op, const void* plan_ws, long E, long num_nodes, int nmax,
                                   const int* nvalid, const void* W, const void* R, const float* bias, void* msg_ws,
                                   float* root_ws, int mode, const float* xres, const float* cscale, float* out_f,
                                   void* out_t, void* stream) {
    using namespace fpm;
    FPM_CHECK_ARG(dtype == 0 || dtype == 1, "spline_conv: bad dtype");
    FPM_CHECK_ARG(mode == 0 || (mode == 1 && xres), "spline_conv: mode 1 needs xres");
    long max_tiles = (E + GBM - 1) / GBM + 25;
    PlanLayout L = plan_layout(E, num_nodes, max_tiles);
    const char* w = (const char*)plan_ws;
    hipStream_t st = (hipStream_t)stream;
    const int D = 768;
    // root term: x R  (fp32 out, bias added after the max like PyG: (max + xR) + b)
    {
        GemmParams p = {};
        p.A = x_op; p.lda = D; p.B = R; p.ldb = D; p.M = (int)num_nodes; p.N = D; p.K = D; p.nseg = 1;
        p.epi = EPI_STORE; p.Cf = root_ws; p.ldc = D;
        dim3 grid(D / GBN, (unsigned)((num_nodes + GBM - 1) / GBM), 1);
        if (dtype == 0) hipLaunchKernelGGL((gemm_kernel<float, false>), grid, dim3(GTHREADS), 0, st, p);
        else hipLaunchKernelGGL((gemm_kernel<bf16_t, false>), grid, dim3(GTHREADS), 0, st, p);
    }
    // edge messages: grouped GEMM, K = 4 segments x 768
    {
        GemmParams p = {};
        p.A = x_op; p.lda = D; p.a_rows = (const int*)(w + L.rows_src);
        p.B = W; p.ldb = D; p.sB_seg = (long)D * D;
        p.row_scale = (const float*)(w + L.rows_basis);
        p.M = (int)E; p.N = D; p.K = D; p.nseg = 4;
        p.tile_info = (const int*)(w + L.tile_info);
        p.group_off = (const int*)(w + L.grp_off);
        p.epi = EPI_STORE; p.Ct = msg_ws; p.ldc = D;
        dim3 grid(D / GBN, (unsigned)max_tiles, 1);
        ProfRec rec = {nullptr, nullptr, 2.0 * (double)E * 4.0 * D * D};
        if (g_prof_on) {
            (void)hipEventCreate(&rec.a);
            (void)hipEventCreate(&rec.b);
            (void)hipEventRecord(rec.a, st);
        }
        if (dtype == 0) hipLaunchKernelGGL((gemm_kernel<float, true>), grid, dim3(GTHREADS), 0, st, p);
        else hipLaunchKernelGGL((gemm_kernel<bf16_t, true>), grid, dim3(GTHREADS), 0, st, p);
        if (g_prof_on) {
            (void)hipEventRecord(rec.b, st);
            g_prof.push_back(rec);
        }
    }
    {
        dim3 grid((unsigned)((num_nodes + 3) / 4));
        if (dtype == 0)
            hipLaunchKernelGGL((segmax_kernel<float>), grid, dim3(256), 0, st, (const float*)msg_ws, root_ws, bias,
                               (const int*)(w + L.dst_ptr), (const int*)(w + L.dst_rows), num_nodes, nmax, nvalid,
                               mode, xres, cscale, out_f, (float*)out_t);
        else
            hipLaunchKernelGGL((segmax_kernel<bf16_t>), grid, dim3(256), 0, st, (const bf16_t*)msg_ws, root_ws, bias,
                               (const int*)(w + L.dst_ptr), (const int*)(w + L.dst_rows), num_nodes, nmax, nvalid,
                               mode, xres, cscale, out_f, (bf16_t*)out_t);
    }
    return check_launch("fpm_spline_conv_fwd");
}

// Xe[e] = x[src] - x[dst]  (vertex_attr_to_edge_attr, spline_conv.py:73-81; feeds only the dead
// edge affinity Ke, computed on request).
namespace {
__global__ void edge_diff_kernel(const float* __restrict__ x, const int* __restrict__ src,
                                 const int* __restrict__ dst, long E, int D, float* __restrict__ out) {
    long e = blockIdx.x;
    if (e >= E) return;
    const float* a = x + (long)src[e] * D;
    const float* b = x + (long)dst[e] * D;
    for (int c = threadIdx.x; c < D; c += blockDim.x) out[e * D + c] = a[c] - b[c];
}
}  // namespace

extern "C" int fpm_edge_diff(const float* x, const int* src, const int* dst, long E, int D, float* out, void* stream) {
    if (E <= 0) return 0;
    hipLaunchKernelGGL(edge_diff_kernel, dim3((unsigned)E), dim3(256), 0, (hipStream_t)stream, x, src, dst, E, D, out);
    return fpm::check_launch("fpm_edge_diff");
}

extern "C" int fpm_profile_enable(int on) {
    g_prof_on = on != 0;
    return 0;
}

// Sum of the recorded edge-GEMM durations (ms) and algorithmic FLOPs since the last read.
extern "C" int fpm_profile_read(double* ms_total, double* flops_total, int* count) {
    double ms = 0.0, fl = 0.0;
    for (auto& r : g_prof) {
        float t = 0.f;
        if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&t, r.a, r.b) != hipSuccess) {
            fpm::set_error("fpm_profile_read: event query failed");
            return 2;
        }
        ms += t;
        fl += r.flops;
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    if (count) *count = (int)g_prof.size();
    g_prof.clear();
    if (ms_total) *ms_total = ms;
    if (flops_total) *flops_total = fl;
    return 0;
}
