// Host (CPU-tensor) halves of the reference's sparse extension ops: the reference runs these on
// the CPU (src/extension/sparse_dot/sparse_dot.cpp:50-140 csr_dot_csc_to_csr, CPU-only there;
// :228-255 csr_dot_diag_to_csr; bilinear_diag.cpp:231-276).  Same storage convention and sums as
// csrc/sparse.hip.  Not on the Net.forward path.
#include <stdint.h>
#include <vector>

namespace fpm {
void set_error(const char* fmt, ...);
}

namespace {

template <typename T>
long csr_dot_csc_csr(const long* i1, const long* p1, const T* d1, const long* i2, const long* p2, const T* d2, long B,
                     long out_h, long out_w, long* out_ptr, long cap, long* out_idx, T* out_data) {
    long nnz = 0;
    if (out_ptr) out_ptr[0] = 0;
    for (long b = 0; b < B; ++b)
        for (long i = 0; i < out_h; ++i) {
            const long rb = p1[b * out_h + i], re = p1[b * out_h + i + 1];
            for (long j = 0; j < out_w; ++j) {
                long a = rb, q = p2[b * out_w + j];
                const long qe = p2[b * out_w + j + 1];
                T acc = (T)0;
                while (a < re && q < qe) {
                    if (i1[a] == i2[q]) {
                        acc += d1[a] * d2[q];
                        ++a;
                        ++q;
                    } else if (i1[a] < i2[q]) {
                        ++a;
                    } else {
                        ++q;
                    }
                }
                if (acc != (T)0) {
                    if (out_idx && nnz < cap) {
                        out_idx[nnz] = j;
                        out_data[nnz] = acc;
                    }
                    ++nnz;
                }
            }
            if (out_ptr) out_ptr[b * out_h + i + 1] = nnz;
        }
    return nnz;
}

template <typename T>
void csr_dot_diag(const long* i1, const long* p1, const T* d1, const T* t2, long B, long out_h, long out_w, T* out) {
    for (long b = 0; b < B; ++b)
        for (long i = 0; i < out_h; ++i)
            for (long q = p1[b * out_h + i]; q < p1[b * out_h + i + 1]; ++q) out[q] = d1[q] * t2[b * out_w + i1[q]];
}

template <typename T>
void bilinear_diag(const long* i1, const long* p1, const T* d1, const T* t2, long feat, const long* i3, const long* p3,
                   const T* d3, long B, long xlen, T* out) {
    for (long b = 0; b < B; ++b)
        for (long i = 0; i < xlen; ++i) {
            const long s = b * xlen + i;
            T acc = (T)0;
            for (long p = p1[s]; p < p1[s + 1]; ++p)
                for (long q = p3[s]; q < p3[s + 1]; ++q) acc += t2[(b * feat + i1[p]) * feat + i3[q]] * d1[p] * d3[q];
            out[s] = acc;
        }
}

}  // namespace

extern "C" {

// Two-call protocol: with out_indices == NULL only the nnz is returned (and out_indptr filled if
// given); then call again with buffers of capacity >= nnz.  Returns nnz, or -1 on a bad dtype.
long fpm_csr_dot_csc_to_csr_host(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                                 const long* t2_indices, const long* t2_indptr, const void* t2_data, long batch_size,
                                 long out_h, long out_w, long* out_indptr, long capacity, long* out_indices,
                                 void* out_data) {
    if (dtype == 0)
        return csr_dot_csc_csr(t1_indices, t1_indptr, (const float*)t1_data, t2_indices, t2_indptr,
                               (const float*)t2_data, batch_size, out_h, out_w, out_indptr, capacity, out_indices,
                               (float*)out_data);
    if (dtype == 2)
        return csr_dot_csc_csr(t1_indices, t1_indptr, (const double*)t1_data, t2_indices, t2_indptr,
                               (const double*)t2_data, batch_size, out_h, out_w, out_indptr, capacity, out_indices,
                               (double*)out_data);
    fpm::set_error("csr_dot_csc_to_csr_host: dtype %d unsupported (0 f32, 2 f64)", dtype);
    return -1;
}

int fpm_csr_dot_diag_to_csr_host(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                                 const void* t2, long batch_size, long out_h, long out_w, void* out_data) {
    if (dtype == 0)
        csr_dot_diag(t1_indices, t1_indptr, (const float*)t1_data, (const float*)t2, batch_size, out_h, out_w,
                     (float*)out_data);
    else if (dtype == 2)
        csr_dot_diag(t1_indices, t1_indptr, (const double*)t1_data, (const double*)t2, batch_size, out_h, out_w,
                     (double*)out_data);
    else {
        fpm::set_error("csr_dot_diag_to_csr_host: dtype %d unsupported (0 f32, 2 f64)", dtype);
        return 1;
    }
    return 0;
}

int fpm_bilinear_diag_host(int dtype, const long* t1_indices, const long* t1_indptr, const void* t1_data,
                           const void* t2, long feat_size, const long* t3_indices, const long* t3_indptr,
                           const void* t3_data, long batch_size, long xlen, void* out) {
    if (dtype == 0)
        bilinear_diag(t1_indices, t1_indptr, (const float*)t1_data, (const float*)t2, feat_size, t3_indices,
                      t3_indptr, (const float*)t3_data, batch_size, xlen, (float*)out);
    else if (dtype == 2)
        bilinear_diag(t1_indices, t1_indptr, (const double*)t1_data, (const double*)t2, feat_size, t3_indices,
                      t3_indptr, (const double*)t3_data, batch_size, xlen, (double*)out);
    else {
        fpm::set_error("bilinear_diag_host: dtype %d unsupported (0 f32, 2 f64)", dtype);
        return 1;
    }
    return 0;
}

}  // extern "C"
