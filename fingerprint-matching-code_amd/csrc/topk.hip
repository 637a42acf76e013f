// Soft top-k (reference src/model/soft_topk.py:8-53 + Sinkhorn_m.forward_log :166-255) and the
// greedy top-k selector over the Hungarian matches (ngm.py:444-449, soft_topk.py:56-77).
//
// soft top-k: one 1024-thread workgroup per pair; the valid block of ss (n1b*n2b <= 65536) is held
// in VGPRs.  The 2-column Sinkhorn runs in dual form: L[q,c] = D[q,c] - u[q] - v[c] with
// D[q,0] = -|ss_q - min|/tau, D[q,1] = -|ss_q - max|/tau.  u[q] = lse_c(D[q,c] - vu[c]) is a
// function of the column potentials seen at the last row step (vu), so the state is four
// scalars and one pass over q per column step is a whole iteration.  The reference's
// data-dependent ``while any(L > 0)`` continuation is kept (bounded at 64 extra steps).
// Values are kept in log2 units (L2 = L log2 e; the test L > 0 is unit-free), so each exp/log is
// one native v_exp_f32 / v_log_f32.
#include "fpm_common.h"
#include <cstdlib>

namespace {

// log2-unit logsumexp of a row's two entries (one term is exp2(0) = 1 exactly, so u >= max and
// L = a - u <= 0 after a row step, as in the reference).  The max term's exp2(0) = 1 is not
// evaluated: 1 + exp2(min - max) is the same sum in either order (one exp, one log per entry).
__device__ __forceinline__ float urow(float a0, float a1) {
    const float m = fmaxf(a0, a1);
    if (m == -INFINITY) return INFINITY;
    return m + fpm::fast_log2(1.f + fpm::fast_exp2(fminf(a0, a1) - m));
}

// STREAM: blocks beyond 64 values per thread (n1*n2 > 65536, e.g. n = 512) re-read ss from
// L2 / HBM on every pass instead of holding it on chip.
template <int NQ, bool STREAM>
__global__ __launch_bounds__(1024) void soft_topk_kernel(const float* __restrict__ ss, long sb, long ld,
                                                         const int* __restrict__ n1, const int* __restrict__ n2,
                                                         const float* __restrict__ kvec, float* __restrict__ out,
                                                         long ob, long old_, int n1max, int n2max, int iters,
                                                         float tau, int* __restrict__ steps_out,
                                                         float* __restrict__ out2, long ob2, long old2,
                                                         int fast_cols) {
    __shared__ float sa[16], sb_[16];
    __shared__ int sflag[16];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n1b = n1[b], n2b = n2[b];
    const int N = n1b * n2b;
    const float* S = ss + (long)b * sb;

    // values k < NQR stay in VGPRs, the rest in LDS (keeps the 1024-thread block under 128 VGPRs)
    constexpr int NQR = STREAM ? 1 : (NQ < 32 ? NQ : 32);
    constexpr int NQL = STREAM ? 0 : NQ - NQR;
    __shared__ float sl[NQL > 0 ? NQL * 1024 : 1];
    float sr[NQR];
#define SVAL(k) ((k) < NQR ? sr[(k) < NQR ? (k) : 0] : sl[((k) >= NQR ? (k) - NQR : 0) * 1024 + tid])
    float mn = INFINITY, mx = -INFINITY;
    if (STREAM) {
        sr[0] = 0.f;
        for (int q = tid; q < N; q += 1024) {
            const int i = q / n2b, j = q - i * n2b;
            const float v = S[i * ld + j];
            mn = fminf(mn, v);
            mx = fmaxf(mx, v);
        }
    } else {
        // (i, j) of q = tid + 1024 k advanced by 1024 entries per k: one division per thread instead
        // of one per value (a runtime-divisor division is ~20 VALU instructions)
        const int n2s = n2b > 0 ? n2b : 1;
        const int di = 1024 / n2s, dj = 1024 - di * n2s;
        int i = tid / n2s, j = tid - i * n2s;
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            int q = tid + 1024 * k;
            float v = 0.f;
            if (q < N) {
                v = S[i * ld + j];
                mn = fminf(mn, v);
                mx = fmaxf(mx, v);
            }
            if (k < NQR) sr[k < NQR ? k : 0] = v;
            else sl[(k >= NQR ? k - NQR : 0) * 1024 + tid] = v;
            i += di;
            j += dj;
            if (j >= n2s) { j -= n2s; ++i; }
        }
    }
    mn = -fpm::warp_max(-mn);
    mx = fpm::warp_max(mx);
    if (lane == 0) { sa[wv] = mn; sb_[wv] = mx; }
    __syncthreads();
    mn = sa[0]; mx = sb_[0];
    for (int w = 1; w < 16; ++w) { mn = fminf(mn, sa[w]); mx = fmaxf(mx, sb_[w]); }
    __syncthreads();

    // dist_mat = -|s - anchor| (soft_topk.py:28-29), then Sinkhorn_m divides by tau (:180);
    // recomputed from s on every pass (keeps 64 values per thread resident instead of 128)
    const float dscale = fpm::LOG2E_F / tau;   // distances / tau, in log2 units
    // visit every q of this thread: register-resident values (unrolled), then LDS-resident ones
    // (runtime loop: bounded code size and register pressure)
    // f(q, value) with q the flat index i * n2b + j of the valid block.  STREAM: a dense block
    // (ld == n2b, 16-B aligned, N % 4 == 0) is read as float4 quads q = 4 (tid + 1024 t) + 0..3;
    // otherwise (i, j) advance by 1024 entries per step without a division.
    const bool dense4 = STREAM && ld == n2b && (N & 3) == 0 && ((unsigned long)S & 15) == 0;
    auto forq = [&](auto&& f) {
        if (STREAM) {
            if (dense4) {
                const float4* S4 = (const float4*)S;
                for (int t = tid; 4 * t < N; t += 1024) {
                    const float4 v = S4[t];
                    f(4 * t, v.x);
                    f(4 * t + 1, v.y);
                    f(4 * t + 2, v.z);
                    f(4 * t + 3, v.w);
                }
                return;
            }
            const int di = 1024 / n2b, dj = 1024 - di * n2b;
            int i = tid / n2b, j = tid - i * n2b;
            for (int q = tid; q < N; q += 1024) {
                f(q, S[i * ld + j]);
                i += di;
                j += dj;
                if (j >= n2b) { j -= n2b; ++i; }
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < NQR; ++k)
            if (tid + 1024 * k < N) f(tid + 1024 * k, sr[k]);
        for (int k = NQR; k < NQ; ++k)
            if (tid + 1024 * k < N) f(tid + 1024 * k, sl[(k - NQR) * 1024 + tid]);
    };
    const float kk = kvec[b];
    const float lcp0 = fpm::fast_log2((float)N - kk);   // log(col_prob[:,0]) = log(n1*n2 - k)
    const float lcp1 = fpm::fast_log2(kk);              // log(col_prob[:,1]) = log(k)
    // state: L_c(q) = a_c - u(q) [after a row step]  or  ((a_c - u) - lse_c) + lcp_c [after a
    // column step], a_c = D_c - vu_c, u = lse(a_0, a_1).  The last two steps are evaluated with the
    // reference's own operation order, so "L <= 0 after a row step" holds exactly as it does there.
    float vu0 = 0.f, vu1 = 0.f, lse0 = 0.f, lse1 = 0.f;
    int last = 0;   // 0: none, 1: row, 2: column
    // maxima of the last reference-order column step's input (valid while last == 2 after it)
    float cm0 = -INFINITY, cm1 = -INFINITY;
    bool cm_ok = false;

    // opaque copies of the anchors: stops the compiler from hoisting the 2*NQ distances out of
    // the iteration loop (that would need 128 more VGPRs and spill)
    auto anchors = [&](float& lo, float& hi) {
        lo = mn;
        hi = mx;
        asm volatile("" : "+v"(lo), "+v"(hi));
    };
    auto Lpair = [&](float sv, float mnl, float mxl, float& L0, float& L1) {
        float a0 = (-fabsf(sv - mnl)) * dscale - vu0, a1 = (-fabsf(sv - mxl)) * dscale - vu1;
        float u = urow(a0, a1);
        L0 = a0 - u;
        L1 = a1 - u;
        if (last == 2) {
            L0 = (L0 - lse0) + lcp0;
            L1 = (L1 - lse1) + lcp1;
        }
        if (L0 != L0) L0 = -INFINITY;
        if (L1 != L1) L1 = -INFINITY;
    };
    auto rowstep = [&]() {
        if (last == 2) {
            float t0 = vu0 + (lse0 - lcp0), t1 = vu1 + (lse1 - lcp1);
            vu0 = (lse0 == -INFINITY || t0 != t0) ? INFINITY : t0;
            vu1 = (lse1 == -INFINITY || t1 != t1) ? INFINITY : t1;
        }
        last = 1;
        cm_ok = false;
    };
    // fast: one pass shifted by the column's log target instead of a max pass (every entry of a
    // row-normalised L is <= 0, and a column's sum stays within 2^+-30 of its target here; a sum
    // outside that range falls back).  Used for the column steps before the last fixed step, so
    // the value the continuation test reads comes from the reference's max-shifted form.
    auto colstep = [&](bool fast) {   // always follows a row step
        float mnl, mxl;
        // the fast pass needs finite potentials (an infinite one is the reference's NaN -> -inf case)
        if (fast && fabsf(vu0) < INFINITY && fabsf(vu1) < INFINITY) {
            anchors(mnl, mxl);
            // after a row step exp2(L_c) = exp2(a_c - lse(a_0, a_1)) is a two-way softmax of
            // d = a_1 - a_0: with t = exp2(-|d|) the larger entry is 1 / (1 + t), the smaller t / (1 + t),
            // and the two sum to 1, so only the column-1 sum is accumulated (column 0 = N - it).  Every
            // valid value lies in [min, max], so |s - min| - |s - max| = 2 s - min - max and
            // d = 2 s dscale - (min + max) dscale - (vu1 - vu0): one fma per entry.  Eight VALU per
            // entry instead of ~17 (two anchor distances, the -inf test, both sums); the column
            // targets exp2(-lcp_c) factor out of the sums.  Early column steps only (the last fixed
            // step and the continuation use the reference's operation order, below).
            const float d2 = 2.f * dscale, dc = -(mnl + mxl) * dscale - (vu1 - vu0);
            float a1 = 0.f;
            forq([&](int k, float sv) {
                const float d = fmaf(sv, d2, dc);
                const float t = fpm::fast_exp2(-fabsf(d));
                const float r = __builtin_amdgcn_rcpf(1.f + t);
                a1 += d > 0.f ? r : t * r;
            });
            a1 = fpm::warp_sum(a1);
            if (lane == 0) sb_[wv] = a1;
            __syncthreads();
            a1 = 0.f;
            for (int w = 0; w < 16; ++w) a1 += sb_[w];
            __syncthreads();
            float a0 = ((float)N - a1) * fpm::fast_exp2(-lcp0);
            a1 *= fpm::fast_exp2(-lcp1);
            if (a0 >= 0x1p-30f && a0 <= 0x1p30f && a1 >= 0x1p-30f && a1 <= 0x1p30f) {
                lse0 = lcp0 + fpm::fast_log2(a0);
                lse1 = lcp1 + fpm::fast_log2(a1);
                last = 2;
                cm_ok = false;
                return;
            }
        }
        anchors(mnl, mxl);
        float m0 = -INFINITY, m1 = -INFINITY;
        forq([&](int k, float sv) {
            float L0, L1;
            Lpair(sv, mnl, mxl, L0, L1);
            m0 = fmaxf(m0, L0);
            m1 = fmaxf(m1, L1);
        });
        m0 = fpm::warp_max(m0);
        m1 = fpm::warp_max(m1);
        if (lane == 0) { sa[wv] = m0; sb_[wv] = m1; }
        __syncthreads();
        m0 = sa[0]; m1 = sb_[0];
        for (int w = 1; w < 16; ++w) { m0 = fmaxf(m0, sa[w]); m1 = fmaxf(m1, sb_[w]); }
        __syncthreads();
        float a0 = 0.f, a1 = 0.f;
        anchors(mnl, mxl);   // fresh opaque anchors: recompute L instead of keeping 2*NQ values live
        forq([&](int k, float sv) {
            float L0, L1;
            Lpair(sv, mnl, mxl, L0, L1);
            if (m0 != -INFINITY) a0 += fpm::fast_exp2(L0 - m0);
            if (m1 != -INFINITY) a1 += fpm::fast_exp2(L1 - m1);
        });
        a0 = fpm::warp_sum(a0);
        a1 = fpm::warp_sum(a1);
        if (lane == 0) { sa[wv] = a0; sb_[wv] = a1; }
        __syncthreads();
        a0 = 0.f; a1 = 0.f;
        for (int w = 0; w < 16; ++w) { a0 += sa[w]; a1 += sb_[w]; }
        __syncthreads();
        lse0 = (m0 == -INFINITY) ? -INFINITY : m0 + fpm::fast_log2(a0);
        lse1 = (m1 == -INFINITY) ? -INFINITY : m1 + fpm::fast_log2(a1);
        last = 2;
        cm0 = m0;
        cm1 = m1;
        cm_ok = true;
    };
    // any(L > 0) (soft_topk.py:232).  After a row step (or none) every L = a - u <= 0 exactly (u >=
    // max(a_0, a_1) in rounded arithmetic): false without a pass.  After a reference-order column
    // step L_c = (x - lse_c) + lcp_c is monotone in x (rounding is monotone), so its maximum is the
    // one at x = the step's own maximum cm_c: the test is two scalar comparisons, the same verdict
    // as the pass over every entry.
    auto any_pos = [&]() -> bool {
        if (last != 2) return false;
        if (cm_ok) {
            const bool p0 = cm0 != -INFINITY && ((cm0 - lse0) + lcp0) > 0.f;
            const bool p1 = cm1 != -INFINITY && ((cm1 - lse1) + lcp1) > 0.f;
            return p0 || p1;
        }
        float mnl, mxl;
        anchors(mnl, mxl);
        int flag = 0;
        forq([&](int k, float sv) {
            float L0, L1;
            Lpair(sv, mnl, mxl, L0, L1);
            flag |= (L0 > 0.f) | (L1 > 0.f);
        });
        int wf = __any(flag) ? 1 : 0;
        if (lane == 0) sflag[wv] = wf;
        __syncthreads();
        int r = 0;
        for (int w = 0; w < 16; ++w) r |= sflag[w];
        __syncthreads();
        return r != 0;
    };

    int step = 0;
    for (; step < iters; ++step) {
        if (step & 1) colstep(fast_cols && step + 2 < iters);
        else rowstep();
    }
    for (int guard = 0; guard < 64 && any_pos(); ++guard, ++step) {
        if (step & 1) colstep(false);
        else rowstep();
    }
    if (steps_out && tid == 0) steps_out[b] = step;

    // ds_mat[i][j] = exp(L[q(i,j), 1]) on the valid block, 0 elsewhere
    float* O = out + (long)b * ob;
    float* O2 = out2 ? out2 + (long)b * ob2 : nullptr;   // optional second copy (host-mapped pinned memory)
    float mnl, mxl;
    anchors(mnl, mxl);
    if (n1b < n1max || n2b < n2max) {   // zero the padding (division-free (i, j) walk)
        const int di = 1024 / n2max, dj = 1024 - di * n2max;
        int i = tid / n2max, j = tid - i * n2max;
        for (int idx = tid; idx < n1max * n2max; idx += 1024) {
            if (i >= n1b || j >= n2b) {
                O[i * old_ + j] = 0.f;
                if (O2) O2[i * old2 + j] = 0.f;
            }
            i += di;
            j += dj;
            if (j >= n2max) { j -= n2max; ++i; }
        }
    }
    int n2o = n2b > 0 ? n2b : 1;
    asm volatile("" : "+v"(n2o));   // recompute (i, j) here rather than keep NQ addresses live
    // forq visits q = tid + 1024 k in ascending k (register values, then LDS values; the STREAM
    // walks pass their own q): (i, j) advanced per visit, one division per thread
    const int dio = 1024 / n2o, djo = 1024 - dio * n2o;
    int io = tid / n2o, jo = tid - io * n2o;
    forq([&](int q, float sv) {
        int i, j;
        if (STREAM) {
            i = q / n2o;
            j = q - i * n2o;
        } else {
            i = io;
            j = jo;
            io += dio;
            jo += djo;
            if (jo >= n2o) { jo -= n2o; ++io; }
        }
        float L0, L1;
        Lpair(sv, mnl, mxl, L0, L1);
        const float v = fpm::fast_exp2(L1);
        O[i * old_ + j] = v;
        if (O2) O2[i * old2 + j] = v;
    });
#undef SVAL
}

// largest n1max / n2max of the selection kernels (the Sinkhorn / soft top-k bound)
constexpr int kSelMax = 2048;

// Greedy top-k over Hungarian matches: prod = x * ds; argsort(prod, desc); accept (r,c) while
// row r and column c are free until round(k) (half-to-even) are accepted.  Positive entries are
// exactly the matched ones (pairwise row/col disjoint), taken in descending value; the
// zero-valued tie region is scanned in ascending flat index (stable order, quirk A.10(v)).
__global__ __launch_bounds__(256) void topk_select_kernel(const float* __restrict__ ds, long sb, long ld,
                                                          const int* __restrict__ assign, long asb,
                                                          const float* __restrict__ kvec, int n1max, int n2max,
                                                          float* __restrict__ perm, long pb, long pld,
                                                          float* __restrict__ lsa_out, long lb, long lld,
                                                          int prezeroed) {
    __shared__ float val[kSelMax];
    __shared__ int key[kSelMax];
    __shared__ unsigned char rowt[kSelMax], colt[kSelMax];
    const int b = blockIdx.x, tid = threadIdx.x;
    const float* D = ds + (long)b * sb;
    const int* A = assign + (long)b * asb;
    float* P = perm + (long)b * pb;
    // zero both outputs: 16-B stores over dense blocks, row-wise (no division) otherwise
    auto zero_block = [&](float* Z, long zld) {
        if (zld == n2max && (n2max & 3) == 0 && ((unsigned long)Z & 15) == 0) {
            float4* Z4 = (float4*)Z;
            const long n4 = (long)n1max * n2max / 4;
            for (long t = tid; t < n4; t += 256) Z4[t] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            for (int i = 0; i < n1max; ++i)
                for (int j = tid; j < n2max; j += 256) Z[i * zld + j] = 0.f;
        }
    };
    if (!prezeroed) {
        zero_block(P, pld);
        if (lsa_out) zero_block(lsa_out + (long)b * lb, lld);
    }
    for (int r = tid; r < kSelMax; r += 256) { rowt[r] = 0; colt[r] = 0; }
    int n = 1;
    while (n < n1max) n <<= 1;
    for (int r = tid; r < n; r += 256) {
        float v = -1.f;
        int kq = 0x7fffffff;
        if (r < n1max) {
            int c = A[r];
            if (c >= 0) {
                v = D[r * ld + c];
                kq = r * n2max + c;
            }
        }
        val[r] = v;
        key[r] = kq;
    }
    __syncthreads();
    if (lsa_out) {
        for (int r = tid; r < n1max; r += 256) {
            int c = A[r];
            if (c >= 0) lsa_out[(long)b * lb + r * lld + c] = 1.f;
        }
    }
    // The positive candidates are the assignment's matches (one per row, distinct columns), so the
    // greedy walk over them in (value desc, flat index asc) order accepts the first K of them: a
    // match is taken iff its rank in that order is < K.  Ranks by direct counting (each thread one
    // or more rows against all n entries, LDS broadcast reads) instead of a bitonic sort and a
    // serial walk; the zero-valued region (fewer than K positive matches) keeps the serial fill.
    const int K = (int)rintf(kvec[b]);
    __shared__ int nacc_s;
    if (tid == 0) nacc_s = 0;
    __syncthreads();
    for (int r = tid; r < n1max; r += 256) {
        const float v = val[r];
        if (!(v > 0.f)) continue;
        const int kr = key[r];
        int rank = 0;
        for (int t = 0; t < n1max; ++t) {
            const float u = val[t];
            rank += (u > v) || (u == v && key[t] < kr);
        }
        if (rank < K) {
            const int c = kr - r * n2max;
            rowt[r] = 1;
            colt[c] = 1;
            P[r * pld + c] = 1.f;
            atomicAdd(&nacc_s, 1);
        }
    }
    __syncthreads();
    // zero-valued region (fewer than K positive matches): the serial walk pairs the i-th free row
    // with the i-th free column (both ascending) until K are taken -- done by one wave with ballot
    // prefix counts (free columns listed in key[], no longer needed)
    const int need = K - nacc_s;
    if (need > 0 && tid < 64) {
        const unsigned long long lt = (1ull << tid) - 1ull;
        int nfc = 0;
        for (int c0 = 0; c0 < n2max; c0 += 64) {
            const int c = c0 + tid;
            const bool f = c < n2max && !colt[c];
            const unsigned long long m = __ballot(f);
            if (f) key[nfc + __popcll(m & lt)] = c;
            nfc += __popcll(m);
        }
        const int take = need < nfc ? need : nfc;
        int i0 = 0;
        for (int r0 = 0; r0 < n1max && i0 < take; r0 += 64) {
            const int r = r0 + tid;
            const bool f = r < n1max && !rowt[r];
            const unsigned long long m = __ballot(f);
            const int i = i0 + __popcll(m & lt);
            if (f && i < take) P[r * pld + key[i]] = 1.f;
            i0 += __popcll(m);
        }
    }
    (void)n;
}


// greedy_perm(x, top_indices, ks) (soft_topk.py:56-77) for an arbitrary candidate order: walk
// top_indices[b][0..T) and accept (row, col) = (idx / n2max, idx % n2max) while the row and the
// column of x still sum to < 1, until round(ks[b]) (half-to-even) are accepted.  x is updated in
// place like the reference's; its initial row / column sums are taken into account.  One
// workgroup per pair: the sums are built in parallel, the walk is serial (it is order dependent)
// with the next 256 candidates staged in LDS.
__global__ __launch_bounds__(256) void greedy_perm_kernel(const long* __restrict__ top, long tsb, int T,
                                                          const float* __restrict__ kvec, int n1max, int n2max,
                                                          float* __restrict__ x, long xb, long xld) {
    __shared__ float rows[kSelMax], cols[kSelMax];
    __shared__ long cand[256];
    __shared__ int done;
    const int b = blockIdx.x, tid = threadIdx.x;
    float* X = x + (long)b * xb;
    for (int r = tid; r < n1max; r += 256) {
        float a = 0.f;
        for (int c = 0; c < n2max; ++c) a += X[r * xld + c];
        rows[r] = a;
    }
    for (int c = tid; c < n2max; c += 256) {
        float a = 0.f;
        for (int r = 0; r < n1max; ++r) a += X[r * xld + c];
        cols[c] = a;
    }
    if (tid == 0) done = 0;
    __syncthreads();
    const int K = (int)rintf(kvec[b]);
    int matched = 0;                      // meaningful in thread 0 only
    for (int t0 = 0; t0 < T; t0 += 256) {
        if (tid < 256 && t0 + tid < T) cand[tid] = top[(long)b * tsb + t0 + tid];
        __syncthreads();
        if (tid == 0) {
            const int tn = min(256, T - t0);
            for (int t = 0; t < tn && matched < K; ++t) {
                const long q = cand[t];
                const long r = q / n2max, c = q - r * n2max;
                if (q < 0 || r >= n1max) continue;
                if (cols[c] < 1.f && rows[r] < 1.f) {
                    const float old = X[r * xld + c];
                    X[r * xld + c] = 1.f;
                    rows[r] += 1.f - old;
                    cols[c] += 1.f - old;
                    ++matched;
                }
            }
            if (matched >= K) done = 1;
        }
        __syncthreads();
        if (done) break;
    }
}

}  // namespace

// single-pass early column steps (env FPM_TOPK_FAST / fpm_set_tuning("topk_fast"))
int& soft_topk_fast_flag() {
    static int v = [] {
        const char* e = getenv("FPM_TOPK_FAST");
        return e ? atoi(e) : 1;
    }();
    return v;
}

extern "C" int fpm_soft_topk_fwd(const float* ss, long s_sb, long s_ld, const int* n1, const int* n2,
                                 const float* k, int B, int n1max, int n2max, int iters, float tau,
                                 float* out, long o_sb, long o_ld, int* steps_out, float* out2, long o2_sb,
                                 long o2_ld, void* stream) {
    FPM_CHECK_ARG(B >= 0 && n1max > 0 && n2max > 0, "soft_topk: bad sizes");
    long nn = (long)n1max * n2max;
    FPM_CHECK_ARG(nn <= (1L << 24), "soft_topk: n1max*n2max=%ld too large", nn);
    if (B == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
#define LAUNCH(NQ, ST) hipLaunchKernelGGL((soft_topk_kernel<NQ, ST>), dim3(B), dim3(1024), 0, st, ss, s_sb, s_ld, \
                                           n1, n2, k, out, o_sb, o_ld, n1max, n2max, iters, tau, steps_out, \
                                           out2, o2_sb, o2_ld, fast)
    const int fast = soft_topk_fast_flag();
    if (nn <= 1024) LAUNCH(1, false);
    else if (nn <= 4096) LAUNCH(4, false);
    else if (nn <= 16384) LAUNCH(16, false);
    else if (nn <= 65536) LAUNCH(64, false);
    else LAUNCH(1, true);
#undef LAUNCH
    return fpm::check_launch("fpm_soft_topk_fwd");
}

namespace {
__global__ __launch_bounds__(256) void zero2_kernel(float4* __restrict__ a, float4* __restrict__ b, long n4) {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < n4; k += (long)gridDim.x * 256) {
        a[k] = z;
        if (b) b[k] = z;
    }
}
}  // namespace

extern "C" int fpm_topk_select(const float* ds, long d_sb, long d_ld, const int* assign, long a_sb,
                               const float* k, int B, int n1max, int n2max, float* perm, long p_sb, long p_ld,
                               float* lsa_out, long l_sb, long l_ld, void* stream) {
    FPM_CHECK_ARG(n1max > 0 && n2max > 0 && n1max <= kSelMax && n2max <= kSelMax,
                  "topk_select: 0 < n1max, n2max <= %d required (got %d, %d)", kSelMax, n1max, n2max);
    if (B == 0) return 0;
    // dense outputs: one wide fill of the whole batch range first (a workgroup per pair zeroing its
    // 2 x n1max x n2max floats left half the CUs issuing stores: ~1 TB/s)
    const long box = (long)n1max * n2max;
    const bool dense = p_ld == n2max && p_sb == box && (!lsa_out || (l_ld == n2max && l_sb == box));
    hipStream_t st = (hipStream_t)stream;
    if (dense) {
        // one wide 16-B-store fill of both outputs (the runtime's fill ran at ~0.9 TB/s, twice)
        const long n4 = (long)B * box / 4;
        const bool v4 = ((long)B * box) % 4 == 0 && ((uintptr_t)perm & 15) == 0 && (!lsa_out || ((uintptr_t)lsa_out & 15) == 0);
        if (v4) {
            const long blocks = (n4 + 255) / 256 < 8192 ? (n4 + 255) / 256 : 8192;
            hipLaunchKernelGGL(zero2_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (float4*)perm, (float4*)lsa_out, n4);
        } else {
            (void)hipMemsetAsync(perm, 0, (size_t)B * box * sizeof(float), st);
            if (lsa_out) (void)hipMemsetAsync(lsa_out, 0, (size_t)B * box * sizeof(float), st);
        }
    }
    hipLaunchKernelGGL(topk_select_kernel, dim3(B), dim3(256), 0, st, ds, d_sb, d_ld, assign, a_sb, k, n1max, n2max,
                       perm, p_sb, p_ld, lsa_out, l_sb, l_ld, dense ? 1 : 0);
    return fpm::check_launch("fpm_topk_select");
}

extern "C" int fpm_greedy_perm(const long* top_idx, long t_sb, int T, const float* k, int B, int n1max, int n2max,
                               float* x, long x_sb, long x_ld, void* stream) {
    FPM_CHECK_ARG(B >= 0 && T >= 0 && n1max > 0 && n2max > 0 && n1max <= kSelMax && n2max <= kSelMax,
                  "greedy_perm: 0 < n1max, n2max <= %d required (got %d, %d)", kSelMax, n1max, n2max);
    if (B == 0) return 0;
    hipLaunchKernelGGL(greedy_perm_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, top_idx, t_sb, T, k, n1max,
                       n2max, x, x_sb, x_ld);
    return fpm::check_launch("fpm_greedy_perm");
}
