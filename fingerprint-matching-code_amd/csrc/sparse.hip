// Batched CSR / CSC sparse products: device twins of the reference's pybind extension ops
// (src/extension/sparse_dot/sparse_dot.cpp:322-331 and bilinear_diag.cpp:324-326), used by the
// dense factorized-graph-matching rebuild (utils/factorize_graph_matching.py:140-186) and its
// backward (src/sparse.py:182-235).  Off the live Net.forward path (ngm.py:293-315 is commented
// out); kept for API parity and the small-n cross-check of the Kronecker pattern.
//
// Storage convention (src/sparse_torch/csx_matrix.py:20-93): one indptr of length B*rows+1 (CSR)
// or B*cols+1 (CSC) holding GLOBAL offsets into indices/data (int64), batch b's compressed slot s
// at indptr[b*len + s].  Products accumulate in the data type, in ascending index order along
// the merge of the two compressed lists (the reference's loop order), so sorted duplicate-free
// inputs give the reference's sums exactly.
//
// MI355X layout: one wave per output row; the row's (index, value) list is staged in LDS once and
// every lane merges it against a different column list (csr x csc), so the row is read from HBM
// once instead of once per output element.
#include "fpm_common.h"

namespace {

enum : int { DT_F32 = 0, DT_F64 = 2, DT_F16 = 3 };

constexpr int ROW_CAP = 512;   // row entries staged in LDS per pass (longer rows: several passes)

// out[b,i,j] = sum over matching k of t1[b](i,k) * t2[b](k,j)
template <typename T>
__global__ __launch_bounds__(256) void csr_dot_csc_dense_kernel(const long* __restrict__ i1, const long* __restrict__ p1,
                                                                const T* __restrict__ d1, const long* __restrict__ i2,
                                                                const long* __restrict__ p2, const T* __restrict__ d2,
                                                                long out_h, long out_w, T* __restrict__ out) {
    __shared__ long sidx[4][ROW_CAP];
    __shared__ T sval[4][ROW_CAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long b = blockIdx.y;
    const long i = (long)blockIdx.x * 4 + w;
    if (i >= out_h) return;
    const long rb = p1[b * out_h + i], re = p1[b * out_h + i + 1];
    T* orow = out + (b * out_h + i) * out_w;
    // partial sums carried across passes: a pass covers row entries [c0, c1); column merge resumes
    // at the first column entry whose index is >= the pass's first row index (sorted lists).
    for (long j = lane; j < out_w; j += 64) orow[j] = (T)0;
    for (long c0 = rb; c0 < re; c0 += ROW_CAP) {
        const long c1 = c0 + ROW_CAP < re ? c0 + ROW_CAP : re;
        const int n = (int)(c1 - c0);
        for (int t = lane; t < n; t += 64) {
            sidx[w][t] = i1[c0 + t];
            sval[w][t] = d1[c0 + t];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's own LDS slice: wave-level sync
        __builtin_amdgcn_wave_barrier();
        const long kfirst = sidx[w][0], klast = sidx[w][n - 1];
        for (long j = lane; j < out_w; j += 64) {
            const long cb = p2[b * out_w + j], ce = p2[b * out_w + j + 1];
            T acc = orow[j];
            int a = 0;
            for (long q = cb; q < ce && a < n;) {
                const long k2 = i2[q];
                if (k2 < kfirst) { ++q; continue; }
                if (k2 > klast) break;
                const long k1 = sidx[w][a];
                if (k1 == k2) {
                    acc += sval[w][a] * d2[q];
                    ++a;
                    ++q;
                } else if (k1 < k2) {
                    ++a;
                } else {
                    ++q;
                }
            }
            orow[j] = acc;
        }
        __builtin_amdgcn_wave_barrier();    // all lanes done with this pass's slice before it is refilled
    }
}

// out[b,i,j] = sum_k t1[b,i,k] * t2[b](k,j), t1 dense (B, out_h, t1_w) row-major
template <typename T>
__global__ __launch_bounds__(256) void dense_dot_csc_dense_kernel(const T* __restrict__ t1, const long* __restrict__ i2,
                                                                  const long* __restrict__ p2, const T* __restrict__ d2,
                                                                  long out_h, long out_w, long t1_w,
                                                                  T* __restrict__ out) {
    const long b = blockIdx.y;
    const long ij = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (ij >= out_h * out_w) return;
    const long i = ij / out_w, j = ij - i * out_w;
    const T* row = t1 + (b * out_h + i) * t1_w;
    const long cb = p2[b * out_w + j], ce = p2[b * out_w + j + 1];
    T acc = (T)0;
    long cursor = 0;   // next dense column the merge may match (entries below it are skipped)
    for (long q = cb; q < ce; ++q) {
        const long k = i2[q];
        if (k >= t1_w) break;
        if (k < cursor) continue;
        acc += row[k] * d2[q];
        cursor = k + 1;
    }
    out[(b * out_h + i) * out_w + j] = acc;
}

// data'[nnz in row (b,i)] = data * t2[b, column index]
template <typename T>
__global__ void csr_dot_diag_kernel(const long* __restrict__ i1, const long* __restrict__ p1, const T* __restrict__ d1,
                                    const T* __restrict__ t2, long out_h, long out_w, T* __restrict__ out) {
    const long b = blockIdx.y;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= out_h) return;
    const long rb = p1[b * out_h + i], re = p1[b * out_h + i + 1];
    for (long q = rb; q < re; ++q) out[q] = d1[q] * t2[b * out_w + i1[q]];
}

// out[b,i] = sum_{p in t1 row i} sum_{q in t3 col i} t2[b, idx1[p], idx3[q]] * d1[p] * d3[q]
template <typename T>
__global__ void bilinear_diag_kernel(const long* __restrict__ i1, const long* __restrict__ p1, const T* __restrict__ d1,
                                     const T* __restrict__ t2, long feat, const long* __restrict__ i3,
                                     const long* __restrict__ p3, const T* __restrict__ d3, long xlen,
                                     T* __restrict__ out) {
    const long b = blockIdx.y;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= xlen) return;
    const long s = b * xlen + i;
    const long ab = p1[s], ae = p1[s + 1], cb = p3[s], ce = p3[s + 1];
    const T* m = t2 + b * feat * feat;
    T acc = (T)0;
    for (long p = ab; p < ae; ++p) {
        const T* mrow = m + i1[p] * feat;
        const T v1 = d1[p];
        for (long q = cb; q < ce; ++q) acc += mrow[i3[q]] * v1 * d3[q];
    }
    out[s] = acc;
}

template <typename F>
int dispatch(int dtype, const char* what, F&& f) {
    switch (dtype) {
        case DT_F32: f((float)0); break;
        case DT_F64: f((double)0); break;
        case DT_F16: f((_Float16)0); break;
        default: fpm::set_error("%s: unsupported dtype code %d (0 f32, 2 f64, 3 f16)", what, dtype); return 1;
    }
    return fpm::check_launch(what);
}

}  // namespace

extern "C" int fpm_csr_dot_csc_to_dense(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                                        const long* t2_indices, const long* t2_indptr, const void* t2_data,
                                        long batch_size, long out_h, long out_w, void* out, void* stream) {
    FPM_CHECK_ARG(batch_size >= 0 && out_h >= 0 && out_w >= 0, "csr_dot_csc_to_dense: bad sizes");
    if (batch_size == 0 || out_h == 0 || out_w == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    return dispatch(dtype, "fpm_csr_dot_csc_to_dense", [&](auto z) {
        using T = decltype(z);
        dim3 grid((unsigned)((out_h + 3) / 4), (unsigned)batch_size);
        hipLaunchKernelGGL(csr_dot_csc_dense_kernel<T>, grid, dim3(256), 0, st, t1_indices, t1_indptr,
                           (const T*)t1_data, t2_indices, t2_indptr, (const T*)t2_data, out_h, out_w, (T*)out);
    });
}

extern "C" int fpm_dense_dot_csc_to_dense(int dtype, const void* t1, const long* t2_indices, const long* t2_indptr,
                                          const void* t2_data, long batch_size, long out_h, long out_w, long t1_w,
                                          void* out, void* stream) {
    FPM_CHECK_ARG(batch_size >= 0 && out_h >= 0 && out_w >= 0 && t1_w >= 0, "dense_dot_csc_to_dense: bad sizes");
    if (batch_size == 0 || out_h == 0 || out_w == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    return dispatch(dtype, "fpm_dense_dot_csc_to_dense", [&](auto z) {
        using T = decltype(z);
        dim3 grid((unsigned)((out_h * out_w + 255) / 256), (unsigned)batch_size);
        hipLaunchKernelGGL(dense_dot_csc_dense_kernel<T>, grid, dim3(256), 0, st, (const T*)t1, t2_indices, t2_indptr,
                           (const T*)t2_data, out_h, out_w, t1_w, (T*)out);
    });
}

extern "C" int fpm_csr_dot_diag_to_csr(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                                       const void* t2, long batch_size, long out_h, long out_w, void* out_data,
                                       void* stream) {
    FPM_CHECK_ARG(batch_size >= 0 && out_h >= 0 && out_w >= 0, "csr_dot_diag_to_csr: bad sizes");
    if (batch_size == 0 || out_h == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    return dispatch(dtype, "fpm_csr_dot_diag_to_csr", [&](auto z) {
        using T = decltype(z);
        dim3 grid((unsigned)((out_h + 255) / 256), (unsigned)batch_size);
        hipLaunchKernelGGL(csr_dot_diag_kernel<T>, grid, dim3(256), 0, st, t1_indices, t1_indptr, (const T*)t1_data,
                           (const T*)t2, out_h, out_w, (T*)out_data);
    });
}

extern "C" int fpm_bilinear_diag(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                                 const void* t2, long feat_size, const long* t3_indices, const long* t3_indptr,
                                 const void* t3_data, long batch_size, long xlen, void* out, void* stream) {
    FPM_CHECK_ARG(batch_size >= 0 && xlen >= 0 && feat_size >= 0, "bilinear_diag: bad sizes");
    if (batch_size == 0 || xlen == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    return dispatch(dtype, "fpm_bilinear_diag", [&](auto z) {
        using T = decltype(z);
        dim3 grid((unsigned)((xlen + 255) / 256), (unsigned)batch_size);
        hipLaunchKernelGGL(bilinear_diag_kernel<T>, grid, dim3(256), 0, st, t1_indices, t1_indptr, (const T*)t1_data,
                           (const T*)t2, feat_size, t3_indices, t3_indptr, (const T*)t3_data, xlen, (T*)out);
    });
}
