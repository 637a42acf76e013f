// Host-only sanitizer driver for the C-ABI's CPU code (SURVEY §5 "race detection / sanitizers"):
// csrc/lsa.cpp (the batched LSAP pool, std::thread + AVX-512 paths) and csrc/sparse_host.cpp (the
// host twins of src/extension/sparse_dot/sparse_dot.cpp:50-283 and bilinear_diag.cpp:231-276),
// built with -fsanitize=address,undefined by `build.py --asan` and run by tests/test_asan_host.py
// (once per solver path: FPM_LSA_SCALAR / FPM_LSA_AVX2 / FPM_LSA_DENSE512 / default).
//
// Checks (exit code 0 = all passed; any sanitizer report aborts with a non-zero status):
//   * fpm_lsa_batch_host on random, tie-heavy, rectangular (wide and tall), padded (ld > n2,
//     sb > n1max * ld) and single-row batches, 1 and 8 pool threads, several calls reusing the pool;
//     every assignment is a valid matching whose cost equals a brute-force optimum (n <= 8) and
//     equals the single-thread result bit for bit; NaN input reports the failing pair.
//   * fpm_lsa_submit / fpm_lsa_wait: two batches queued from two threads equal the synchronous result.
//   * the sparse host twins against dense products on random CSR/CSC data (f32 and f64), incl. the
//     two-call protocol of csr_dot_csc_to_csr with an exact and an undersized capacity.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <thread>
#include <vector>

#include "fpm.h"

namespace fpm {
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    fputc('\n', stderr);
}
}  // namespace fpm

static int g_fail = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);              \
            fputc('\n', stderr);                       \
            ++g_fail;                                  \
        }                                              \
    } while (0)

// best total of s over matchings of min(n1, n2) pairs (maximise), by enumeration
static double brute_best(const float* s, long ld, int n1, int n2) {
    const bool tr = n1 > n2;
    const int r = tr ? n2 : n1, c = tr ? n1 : n2;
    std::vector<int> cols(c);
    for (int j = 0; j < c; ++j) cols[j] = j;
    double best = -INFINITY;
    do {
        double t = 0.0;
        for (int i = 0; i < r; ++i) t += tr ? (double)s[(long)cols[i] * ld + i] : (double)s[(long)i * ld + cols[i]];
        best = std::max(best, t);
    } while (std::next_permutation(cols.begin(), cols.end()));
    return best;
}

static void test_lsa(std::mt19937& rng) {
    struct Case {
        int B, n1max, n2max, ld_pad, sb_pad, ties, small;
    };
    const Case cases[] = {{6, 8, 8, 0, 0, 0, 1},   {5, 7, 8, 3, 5, 1, 1},  {4, 8, 6, 0, 0, 1, 1},
                          {16, 64, 64, 1, 0, 0, 0}, {9, 40, 57, 0, 7, 1, 0}, {3, 130, 100, 2, 0, 1, 0},
                          {12, 256, 256, 0, 0, 0, 0}, {2, 1, 5, 0, 0, 0, 1}};
    std::uniform_real_distribution<float> U(0.f, 1.f);
    for (const Case& cs : cases) {
        const long ld = cs.n2max + cs.ld_pad, sb = (long)cs.n1max * ld + cs.sb_pad;
        std::vector<float> s((size_t)sb * cs.B, -7.f);
        std::vector<int> n1(cs.B), n2(cs.B);
        for (int b = 0; b < cs.B; ++b) {
            n1[b] = std::max(1, cs.n1max - (int)(rng() % (cs.small ? 2 : 9)));
            n2[b] = std::max(1, cs.n2max - (int)(rng() % (cs.small ? 2 : 9)));
            for (int i = 0; i < cs.n1max; ++i)
                for (int j = 0; j < cs.n2max; ++j) {
                    float v = U(rng);
                    if (cs.ties) v = floorf(v * 4.f) / 4.f;   // many equal costs
                    s[(size_t)b * sb + (size_t)i * ld + j] = v;
                }
        }
        std::vector<int> a1((size_t)cs.B * cs.n1max, -5), a8((size_t)cs.B * cs.n1max, -5);
        for (int rep = 0; rep < 3; ++rep) {   // the pool is reused across calls
            int rc = fpm_lsa_batch_host(s.data(), sb, ld, n1.data(), n2.data(), cs.B, cs.n1max, a1.data(), 1);
            CHECK(rc == 0, "lsa rc %d (1 thread)", rc);
            rc = fpm_lsa_batch_host(s.data(), sb, ld, n1.data(), n2.data(), cs.B, cs.n1max, a8.data(), 8);
            CHECK(rc == 0, "lsa rc %d (8 threads)", rc);
            CHECK(a1 == a8, "lsa: pool result differs from the single-thread result");
            // the asynchronous queue: two batches in flight from two submitting threads
            std::vector<int> q1((size_t)cs.B * cs.n1max, -5), q2((size_t)cs.B * cs.n1max, -5);
            long t1 = 0, t2 = 0;
            std::thread th([&] { t2 = fpm_lsa_submit(s.data(), sb, ld, n1.data(), n2.data(), cs.B, cs.n1max, q2.data(), 8); });
            t1 = fpm_lsa_submit(s.data(), sb, ld, n1.data(), n2.data(), cs.B, cs.n1max, q1.data(), 8);
            th.join();
            double sec = -1.0;
            rc = fpm_lsa_wait(t2, 1, &sec);
            CHECK(rc == 0 && sec >= 0.0, "lsa async rc %d", rc);
            rc = fpm_lsa_wait(t1, 1, nullptr);
            CHECK(rc == 0, "lsa async rc %d", rc);
            CHECK(fpm_lsa_wait(t1, 1, nullptr) == -1, "lsa async: released ticket still known");
            CHECK(q1 == a1 && q2 == a1, "lsa: async queue result differs from the synchronous one");
        }
        for (int b = 0; b < cs.B; ++b) {
            const int* a = a1.data() + (size_t)b * cs.n1max;
            std::vector<int> used(cs.n2max, 0);
            int m = 0;
            double tot = 0.0;
            for (int i = 0; i < n1[b]; ++i) {
                if (a[i] < 0) continue;
                CHECK(a[i] < n2[b], "lsa: column %d out of range %d", a[i], n2[b]);
                CHECK(!used[a[i]]++, "lsa: column %d assigned twice", a[i]);
                tot += s[(size_t)b * sb + (size_t)i * ld + a[i]];
                ++m;
            }
            CHECK(m == std::min(n1[b], n2[b]), "lsa: %d matches, expected %d", m, std::min(n1[b], n2[b]));
            if (cs.small) {
                const double best = brute_best(s.data() + (size_t)b * sb, ld, n1[b], n2[b]);
                CHECK(fabs(tot - best) <= 1e-5, "lsa: total %.7f, optimum %.7f", tot, best);
            }
        }
    }
    // invalid input: a NaN in pair 1 -> status 2 (pair index + 1)
    std::vector<float> s(3 * 16, 0.5f);
    s[16 + 5] = NAN;
    int n[3] = {4, 4, 4};
    std::vector<int> a(12);
    const int rc = fpm_lsa_batch_host(s.data(), 16, 4, n, n, 3, 4, a.data(), 2);
    CHECK(rc == 2, "lsa: NaN pair reported as %d, expected 2", rc);
}

// random batched CSR (rows x cols) with sorted, duplicate-free indices
template <typename T>
static void rand_csr(std::mt19937& rng, long B, long rows, long cols, double dens, std::vector<long>& ptr,
                     std::vector<long>& idx, std::vector<T>& val, std::vector<T>& dense) {
    std::uniform_real_distribution<double> U(0.0, 1.0);
    ptr.assign(1, 0);
    idx.clear();
    val.clear();
    dense.assign((size_t)B * rows * cols, (T)0);
    for (long b = 0; b < B; ++b)
        for (long r = 0; r < rows; ++r) {
            for (long c = 0; c < cols; ++c)
                if (U(rng) < dens) {
                    const T v = (T)(U(rng) * 2.0 - 1.0);
                    idx.push_back(c);
                    val.push_back(v);
                    dense[((size_t)b * rows + r) * cols + c] = v;
                }
            ptr.push_back((long)idx.size());
        }
}

template <typename T>
static void test_sparse(std::mt19937& rng, int code, double tol) {
    const long B = 3, H = 17, K = 23, W = 19;
    // A: CSR (H x K); Bm as CSC (K x W) = CSR of its transpose (W x K)
    std::vector<long> pa, ia, pb, ib;
    std::vector<T> va, vb, Ad, BTd;
    rand_csr(rng, B, H, K, 0.3, pa, ia, va, Ad);
    rand_csr(rng, B, W, K, 0.3, pb, ib, vb, BTd);
    std::vector<T> ref((size_t)B * H * W, (T)0);
    for (long b = 0; b < B; ++b)
        for (long i = 0; i < H; ++i)
            for (long j = 0; j < W; ++j) {
                T acc = 0;
                for (long k = 0; k < K; ++k) acc += Ad[((size_t)b * H + i) * K + k] * BTd[((size_t)b * W + j) * K + k];
                ref[((size_t)b * H + i) * W + j] = acc;
            }
    // two-call protocol
    std::vector<long> optr(B * H + 1);
    const long nnz = fpm_csr_dot_csc_to_csr_host(code, ia.data(), pa.data(), va.data(), ib.data(), pb.data(), vb.data(),
                                                 B, H, W, optr.data(), 0, nullptr, nullptr);
    CHECK(nnz >= 0, "csr_dot_csc_to_csr: nnz %ld", nnz);
    std::vector<long> oidx(std::max(nnz, 1L));
    std::vector<T> oval(std::max(nnz, 1L));
    const long nnz2 = fpm_csr_dot_csc_to_csr_host(code, ia.data(), pa.data(), va.data(), ib.data(), pb.data(), vb.data(),
                                                  B, H, W, optr.data(), nnz, oidx.data(), oval.data());
    CHECK(nnz2 == nnz, "csr_dot_csc_to_csr: second call nnz %ld vs %ld", nnz2, nnz);
    std::vector<T> got((size_t)B * H * W, (T)0);
    for (long r = 0; r < B * H; ++r)
        for (long q = optr[r]; q < optr[r + 1]; ++q) got[(size_t)r * W + oidx[q]] = oval[q];
    for (size_t e = 0; e < got.size(); ++e)
        CHECK(fabs((double)got[e] - (double)ref[e]) <= tol, "csr_dot_csc_to_csr: entry %zu %g vs %g", e, (double)got[e],
              (double)ref[e]);
    // undersized capacity: the count is still returned, nothing is written past the buffer
    if (nnz > 2) {
        std::vector<long> small_i(2);
        std::vector<T> small_v(2);
        const long n3 = fpm_csr_dot_csc_to_csr_host(code, ia.data(), pa.data(), va.data(), ib.data(), pb.data(),
                                                    vb.data(), B, H, W, optr.data(), 2, small_i.data(), small_v.data());
        CHECK(n3 == nnz, "csr_dot_csc_to_csr: capped call nnz %ld vs %ld", n3, nnz);
    }
    // csr_dot_diag: A (H x K) * diag(t2[b]) -> same pattern
    std::vector<T> t2((size_t)B * K);
    for (auto& v : t2) v = (T)((double)(rng() % 1000) / 500.0 - 1.0);
    std::vector<T> od(va.size() + 1);
    CHECK(fpm_csr_dot_diag_to_csr_host(code, ia.data(), pa.data(), va.data(), t2.data(), B, H, K, od.data()) == 0,
          "csr_dot_diag rc");
    for (long r = 0; r < B * H; ++r)
        for (long q = pa[r]; q < pa[r + 1]; ++q) {
            const T e = va[q] * t2[(r / H) * K + ia[q]];
            CHECK(fabs((double)od[q] - (double)e) <= tol, "csr_dot_diag: %ld", q);
        }
    // bilinear_diag: out[b][i] = sum_{p in row i of A, q in row i of C} t3[b][A.idx[p]][C.idx[q]] A.v C.v
    const long F = K;
    std::vector<long> pc, ic;
    std::vector<T> vc, Cd;
    rand_csr(rng, B, H, F, 0.25, pc, ic, vc, Cd);
    std::vector<T> tt((size_t)B * F * F);
    for (auto& v : tt) v = (T)((double)(rng() % 2000) / 1000.0 - 1.0);
    std::vector<T> ob((size_t)B * H);
    CHECK(fpm_bilinear_diag_host(code, ia.data(), pa.data(), va.data(), tt.data(), F, ic.data(), pc.data(), vc.data(), B,
                                 H, ob.data()) == 0,
          "bilinear_diag rc");
    for (long b = 0; b < B; ++b)
        for (long i = 0; i < H; ++i) {
            double e = 0.0;
            for (long x = 0; x < F; ++x)
                for (long y = 0; y < F; ++y)
                    e += (double)tt[((size_t)b * F + x) * F + y] * (double)Ad[((size_t)b * H + i) * K + x] *
                         (double)Cd[((size_t)b * H + i) * F + y];
            CHECK(fabs((double)ob[b * H + i] - e) <= 10 * tol, "bilinear_diag: (%ld, %ld) %g vs %g", b, i,
                  (double)ob[b * H + i], e);
        }
    // unsupported dtype is an error, not a crash
    CHECK(fpm_csr_dot_diag_to_csr_host(7, ia.data(), pa.data(), va.data(), t2.data(), B, H, K, od.data()) != 0,
          "csr_dot_diag accepted dtype 7");
}

int main() {
    std::mt19937 rng(1234);
    test_lsa(rng);
    test_sparse<float>(rng, 0, 1e-5);
    test_sparse<double>(rng, 2, 1e-12);
    if (g_fail) {
        fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    printf("asan host driver: all checks passed\n");
    return 0;
}
