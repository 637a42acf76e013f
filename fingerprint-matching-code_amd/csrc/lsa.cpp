// Host-side linear sum assignment for utils/hungarian.py:8-66 (scipy.optimize.linear_sum_assignment
// on -s), batched over pairs with a pool of std::threads.
//
// Algorithm: shortest augmenting path with dual potentials (Crouse 2016), the method behind
// scipy >= 1.4's rectangular LSAP solver (scipy 1.10.1 pinned at environment.yml:229).  The
// column scan order (remaining columns filled in reverse), the tie rule (prefer an unassigned
// column among equal reduced costs) and the transpose of tall matrices follow that published
// method so that, on inputs with ties, the same optimum is returned.  Costs are evaluated in
// double from the float32 input (-s), as scipy converts its input to float64.
//
// Third-party notice.  The scalar solver lsap_solve() below restates scipy's
// scipy/optimize/rectangular_lsap/rectangular_lsap.cpp (P. M. Larsen's implementation of Crouse's
// pseudocode) closely, including its variable names; it is kept as the bit-exact reference of the
// vectorised solvers further down.  scipy is distributed under the BSD 3-Clause licence:
//
//   Copyright (c) 2001-2002 Enthought, Inc. 2003, SciPy Developers.
//   All rights reserved.
//
//   Redistribution and use in source and binary forms, with or without modification, are
//   permitted provided that the following conditions are met:
//   1. Redistributions of source code must retain the above copyright notice, this list of
//      conditions and the following disclaimer.
//   2. Redistributions in binary form must reproduce the above copyright notice, this list of
//      conditions and the following disclaimer in the documentation and/or other materials
//      provided with the distribution.
//   3. Neither the name of the copyright holder nor the names of its contributors may be used to
//      endorse or promote products derived from this software without specific prior written
//      permission.
//
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS IS" AND ANY EXPRESS
//   OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE IMPLIED WARRANTIES OF
//   MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE DISCLAIMED. IN NO EVENT SHALL THE
//   COPYRIGHT HOLDER OR CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL,
//   EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE
//   GOODS OR SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED
//   AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING
//   NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF THIS SOFTWARE, EVEN IF ADVISED
//   OF THE POSSIBILITY OF SUCH DAMAGE.
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace {

// returns 0 on success; col4row[i] = assigned column of row i (nr <= nc after transposition)
int lsap_solve(int nr, int nc, const double* cost, std::vector<int>& col4row) {
    std::vector<double> u(nr, 0.0), v(nc, 0.0), spc(nc);
    std::vector<int> path(nc, -1), row4col(nc, -1), remaining(nc);
    std::vector<char> SR(nr), SC(nc);
    col4row.assign(nr, -1);
    for (int cur = 0; cur < nr; ++cur) {
        double minVal = 0.0;
        int i = cur;
        int num_rem = nc;
        for (int it = 0; it < nc; ++it) remaining[it] = nc - it - 1;
        std::fill(SR.begin(), SR.end(), 0);
        std::fill(SC.begin(), SC.end(), 0);
        std::fill(spc.begin(), spc.end(), INFINITY);
        int sink = -1;
        while (sink == -1) {
            int index = -1;
            double lowest = INFINITY;
            SR[i] = 1;
            const double* crow = cost + (long)i * nc;
            const double ui = u[i];
            for (int it = 0; it < num_rem; ++it) {
                const int j = remaining[it];
                const double r = minVal + crow[j] - ui - v[j];
                if (r < spc[j]) {
                    path[j] = i;
                    spc[j] = r;
                }
                if (spc[j] < lowest || (spc[j] == lowest && row4col[j] == -1)) {
                    lowest = spc[j];
                    index = it;
                }
            }
            minVal = lowest;
            if (minVal == INFINITY) return -1;   // infeasible
            const int j = remaining[index];
            if (row4col[j] == -1) sink = j;
            else i = row4col[j];
            SC[j] = 1;
            remaining[index] = remaining[--num_rem];
        }
        u[cur] += minVal;
        for (int r = 0; r < nr; ++r)
            if (SR[r] && r != cur) u[r] += minVal - spc[col4row[r]];
        for (int c = 0; c < nc; ++c)
            if (SC[c]) v[c] -= minVal - spc[c];
        int j = sink;
        while (true) {
            const int r = path[j];
            row4col[j] = r;
            std::swap(col4row[r], j);
            if (r == cur) break;
        }
    }
    return 0;
}

// ---- vectorised form of the same algorithm ------------------------------------------------------
// The remaining columns are kept as structure-of-arrays in the scan order (rc = column id, rs =
// its shortest-path cost, rp = its path row, rv = v[col], ru = column unassigned), so the scan is
// contiguous except for the cost-row gather.  The tie rule of the scalar loop -- index updates on
// spc < lowest, or spc == lowest on an unassigned column -- selects: the last unassigned column
// holding the minimum if there is one, else the first column holding it.  Both forms are the same
// function of the scan order, and the reduced costs are evaluated with the same operation order
// ((minVal + c) - u_i) - v_j, so the result is bit-identical to lsap_solve.
#if defined(__x86_64__)
#include <immintrin.h>

__attribute__((target("avx2"))) int lsap_solve_avx2(int nr, int nc, const double* cost, std::vector<int>& col4row) {
    std::vector<double> u(nr, 0.0), v(nc, 0.0), spc(nc);
    std::vector<int> path(nc, -1), row4col(nc, -1);
    std::vector<char> SR(nr), SC(nc);
    const int ncp = (nc + 3) & ~3;
    std::vector<int> rc(ncp), rp(ncp), ru(ncp);
    std::vector<double> rs(ncp), rv(ncp);
    col4row.assign(nr, -1);
    for (int cur = 0; cur < nr; ++cur) {
        double minVal = 0.0;
        int i = cur;
        int num = nc;
        for (int it = 0; it < nc; ++it) {
            const int j = nc - it - 1;
            rc[it] = j;
            rs[it] = INFINITY;
            rp[it] = -1;
            rv[it] = v[j];
            ru[it] = row4col[j] == -1 ? -1 : 0;
        }
        std::fill(SR.begin(), SR.end(), 0);
        std::fill(SC.begin(), SC.end(), 0);
        int sink = -1;
        while (sink == -1) {
            SR[i] = 1;
            const double* crow = cost + (long)i * nc;
            const double ui = u[i];
            const __m256d vmin = _mm256_set1_pd(minVal), vui = _mm256_set1_pd(ui);
            const __m128i vi = _mm_set1_epi32(i);
            __m256d vlow = _mm256_set1_pd(INFINITY);
            int it = 0;
            for (; it + 4 <= num; it += 4) {
                __m128i cols = _mm_loadu_si128((const __m128i*)&rc[it]);
                __m256d c = _mm256_i32gather_pd(crow, cols, 8);
                __m256d r = _mm256_sub_pd(_mm256_sub_pd(_mm256_add_pd(vmin, c), vui), _mm256_loadu_pd(&rv[it]));
                __m256d sv = _mm256_loadu_pd(&rs[it]);
                __m256d lt = _mm256_cmp_pd(r, sv, _CMP_LT_OQ);
                sv = _mm256_blendv_pd(sv, r, lt);
                _mm256_storeu_pd(&rs[it], sv);
                __m128i m32 = _mm256_cvtpd_epi32(lt);   // all-ones -> -1 lanes? use movemask instead
                (void)m32;
                int mk = _mm256_movemask_pd(lt);
                if (mk) {
                    for (int q = 0; q < 4; ++q)
                        if (mk & (1 << q)) rp[it + q] = i;
                }
                vlow = _mm256_min_pd(vlow, sv);
            }
            (void)vi;
            double lowest;
            {
                double t[4];
                _mm256_storeu_pd(t, vlow);
                lowest = std::min(std::min(t[0], t[1]), std::min(t[2], t[3]));
            }
            for (; it < num; ++it) {
                const double r = minVal + crow[rc[it]] - ui - rv[it];
                if (r < rs[it]) {
                    rs[it] = r;
                    rp[it] = i;
                }
                if (rs[it] < lowest) lowest = rs[it];
            }
            if (lowest == INFINITY) return -1;
            // first position holding the minimum, last unassigned one holding it
            int first = -1, lastu = -1;
            {
                const __m256d vl = _mm256_set1_pd(lowest);
                int q = 0;
                for (; q + 4 <= num; q += 4) {
                    int mk = _mm256_movemask_pd(_mm256_cmp_pd(_mm256_loadu_pd(&rs[q]), vl, _CMP_EQ_OQ));
                    if (mk) {
                        for (int b = 0; b < 4; ++b)
                            if (mk & (1 << b)) {
                                if (first < 0) first = q + b;
                                if (ru[q + b]) lastu = q + b;
                            }
                    }
                }
                for (; q < num; ++q)
                    if (rs[q] == lowest) {
                        if (first < 0) first = q;
                        if (ru[q]) lastu = q;
                    }
            }
            const int index = lastu >= 0 ? lastu : first;
            minVal = lowest;
            const int j = rc[index];
            spc[j] = rs[index];
            path[j] = rp[index];
            if (row4col[j] == -1) sink = j;
            else i = row4col[j];
            SC[j] = 1;
            --num;
            rc[index] = rc[num];
            rs[index] = rs[num];
            rp[index] = rp[num];
            rv[index] = rv[num];
            ru[index] = ru[num];
        }
        u[cur] += minVal;
        for (int r = 0; r < nr; ++r)
            if (SR[r] && r != cur) u[r] += minVal - spc[col4row[r]];
        for (int c = 0; c < nc; ++c)
            if (SC[c]) v[c] -= minVal - spc[c];
        int j = sink;
        while (true) {
            const int r = path[j];
            row4col[j] = r;
            std::swap(col4row[r], j);
            if (r == cur) break;
        }
    }
    return 0;
}
#endif

// ---- dense-scan form (default) -------------------------------------------------------------------
// Same algorithm again, but the Dijkstra scan runs over ALL columns with a "remaining" mask, so
// the cost row, v and spc are read contiguously 4 doubles at a time (no gather, no branches).
// The scan order of the remaining list matters only when several remaining columns hold the
// minimum exactly; then their positions in that list (maintained under the swap-remove) decide,
// with the scalar loop's rule (last unassigned holder of the minimum, else the first holder).
__attribute__((target("avx2"))) int lsap_solve_dense(int nr, int nc, const double* cost, std::vector<int>& col4row) {
    const int ncp = (nc + 3) & ~3;
    std::vector<double> u(nr, 0.0), v(ncp, 0.0), spc(ncp);
    std::vector<long long> rem(ncp);
    std::vector<long long> path(ncp, -1);   // 64-bit so it blends with the double lanes
    std::vector<int> row4col(nc, -1), remaining(nc), pos(nc);
    std::vector<char> SR(nr), SC(nc);
    std::vector<int> ties;
    std::vector<double> crow_pad;
    const bool pad = ncp != nc;
    if (pad) crow_pad.assign(ncp, 0.0);
    col4row.assign(nr, -1);
    const __m256d vinf = _mm256_set1_pd(INFINITY);
    for (int cur = 0; cur < nr; ++cur) {
        double minVal = 0.0;
        int i = cur;
        int num = nc;
        for (int it = 0; it < nc; ++it) {
            remaining[it] = nc - it - 1;
            pos[nc - it - 1] = it;
        }
        for (int j = 0; j < ncp; ++j) {
            rem[j] = j < nc ? -1LL : 0LL;
            spc[j] = INFINITY;
        }
        std::fill(SR.begin(), SR.end(), 0);
        std::fill(SC.begin(), SC.end(), 0);
        int sink = -1;
        while (sink == -1) {
            SR[i] = 1;
            const double* crow = cost + (long)i * nc;
            if (pad) {
                std::copy(crow, crow + nc, crow_pad.begin());
                crow = crow_pad.data();
            }
            const __m256d vmv = _mm256_set1_pd(minVal), vui = _mm256_set1_pd(u[i]);
            const __m256d vi = _mm256_castsi256_pd(_mm256_set1_epi64x(i));
            __m256d vlow = vinf;
            for (int j = 0; j < ncp; j += 4) {
                const __m256d m = _mm256_castsi256_pd(_mm256_loadu_si256((const __m256i*)&rem[j]));
                const __m256d r = _mm256_sub_pd(_mm256_sub_pd(_mm256_add_pd(vmv, _mm256_loadu_pd(crow + j)), vui),
                                                _mm256_loadu_pd(&v[j]));
                __m256d sv = _mm256_loadu_pd(&spc[j]);
                const __m256d lt = _mm256_and_pd(_mm256_cmp_pd(r, sv, _CMP_LT_OQ), m);
                sv = _mm256_blendv_pd(sv, r, lt);
                _mm256_storeu_pd(&spc[j], sv);
                const __m256d pv = _mm256_castsi256_pd(_mm256_loadu_si256((const __m256i*)&path[j]));
                _mm256_storeu_si256((__m256i*)&path[j], _mm256_castpd_si256(_mm256_blendv_pd(pv, vi, lt)));
                vlow = _mm256_min_pd(vlow, _mm256_blendv_pd(vinf, sv, m));
            }
            double t4[4];
            _mm256_storeu_pd(t4, vlow);
            const double lowest = std::min(std::min(t4[0], t4[1]), std::min(t4[2], t4[3]));
            if (lowest == INFINITY) return -1;
            // remaining columns holding the minimum
            ties.clear();
            const __m256d vl = _mm256_set1_pd(lowest);
            for (int j = 0; j < ncp; j += 4) {
                const __m256d m = _mm256_castsi256_pd(_mm256_loadu_si256((const __m256i*)&rem[j]));
                const int mk = _mm256_movemask_pd(_mm256_and_pd(_mm256_cmp_pd(_mm256_loadu_pd(&spc[j]), vl, _CMP_EQ_OQ), m));
                if (mk)
                    for (int q = 0; q < 4; ++q)
                        if (mk & (1 << q)) ties.push_back(j + q);
            }
            int j = ties[0];
            if (ties.size() > 1) {
                int first = -1, lastu = -1, fpos = nc, upos = -1;
                for (int t : ties) {
                    if (pos[t] < fpos) { fpos = pos[t]; first = t; }
                    if (row4col[t] == -1 && pos[t] > upos) { upos = pos[t]; lastu = t; }
                }
                j = lastu >= 0 ? lastu : first;
            }
            minVal = lowest;
            rem[j] = 0;
            const int p = pos[j], last = remaining[--num];
            remaining[p] = last;
            pos[last] = p;
            if (row4col[j] == -1) sink = j;
            else i = row4col[j];
            SC[j] = 1;
        }
        u[cur] += minVal;
        for (int r = 0; r < nr; ++r)
            if (SR[r] && r != cur) u[r] += minVal - spc[col4row[r]];
        for (int c = 0; c < nc; ++c)
            if (SC[c]) v[c] -= minVal - spc[c];
        int j = sink;
        while (true) {
            const int r = (int)path[j];
            row4col[j] = r;
            std::swap(col4row[r], j);
            if (r == cur) break;
        }
    }
    return 0;
}

// Same solver with 8-wide AVX-512 vectors and mask registers (Zen 4/5, Sapphire Rapids hosts).
__attribute__((target("avx512f,avx512dq"))) int lsap_solve_dense512(int nr, int nc, const double* cost,
                                                                   std::vector<int>& col4row) {
    const int ncp = (nc + 7) & ~7;
    std::vector<double> u(nr, 0.0), v(ncp, 0.0), spc(ncp);
    std::vector<long long> rem(ncp);
    std::vector<long long> path(ncp, -1);
    std::vector<int> row4col(nc, -1), remaining(nc), pos(nc);
    std::vector<char> SR(nr), SC(nc);
    std::vector<int> ties;
    std::vector<double> crow_pad;
    const bool pad = ncp != nc;
    if (pad) crow_pad.assign(ncp, 0.0);
    col4row.assign(nr, -1);
    const __m512d vinf = _mm512_set1_pd(INFINITY);
    const __m512i zero = _mm512_setzero_si512();
    for (int cur = 0; cur < nr; ++cur) {
        double minVal = 0.0;
        int i = cur;
        int num = nc;
        for (int it = 0; it < nc; ++it) {
            remaining[it] = nc - it - 1;
            pos[nc - it - 1] = it;
        }
        for (int j = 0; j < ncp; ++j) {
            rem[j] = j < nc ? -1LL : 0LL;
            spc[j] = INFINITY;
        }
        std::fill(SR.begin(), SR.end(), 0);
        std::fill(SC.begin(), SC.end(), 0);
        int sink = -1;
        while (sink == -1) {
            SR[i] = 1;
            const double* crow = cost + (long)i * nc;
            if (pad) {
                std::copy(crow, crow + nc, crow_pad.begin());
                crow = crow_pad.data();
            }
            const __m512d vmv = _mm512_set1_pd(minVal), vui = _mm512_set1_pd(u[i]);
            const __m512i vi = _mm512_set1_epi64(i);
            __m512d vlow = vinf;
            for (int j = 0; j < ncp; j += 8) {
                const __mmask8 m = _mm512_cmpneq_epi64_mask(_mm512_loadu_si512(&rem[j]), zero);
                const __m512d r = _mm512_sub_pd(_mm512_sub_pd(_mm512_add_pd(vmv, _mm512_loadu_pd(crow + j)), vui),
                                                _mm512_loadu_pd(&v[j]));
                __m512d sv = _mm512_loadu_pd(&spc[j]);
                const __mmask8 lt = _mm512_mask_cmp_pd_mask(m, r, sv, _CMP_LT_OQ);
                sv = _mm512_mask_blend_pd(lt, sv, r);
                _mm512_storeu_pd(&spc[j], sv);
                _mm512_mask_storeu_epi64(&path[j], lt, vi);
                vlow = _mm512_mask_min_pd(vlow, m, vlow, sv);
            }
            const double lowest = _mm512_reduce_min_pd(vlow);
            if (lowest == INFINITY) return -1;
            ties.clear();
            const __m512d vl = _mm512_set1_pd(lowest);
            for (int j = 0; j < ncp; j += 8) {
                const __mmask8 m = _mm512_cmpneq_epi64_mask(_mm512_loadu_si512(&rem[j]), zero);
                unsigned mk = _mm512_mask_cmp_pd_mask(m, _mm512_loadu_pd(&spc[j]), vl, _CMP_EQ_OQ);
                while (mk) {
                    const int q = __builtin_ctz(mk);
                    ties.push_back(j + q);
                    mk &= mk - 1;
                }
            }
            int j = ties[0];
            if (ties.size() > 1) {
                int first = -1, lastu = -1, fpos = nc, upos = -1;
                for (int t : ties) {
                    if (pos[t] < fpos) { fpos = pos[t]; first = t; }
                    if (row4col[t] == -1 && pos[t] > upos) { upos = pos[t]; lastu = t; }
                }
                j = lastu >= 0 ? lastu : first;
            }
            minVal = lowest;
            rem[j] = 0;
            const int p = pos[j], last = remaining[--num];
            remaining[p] = last;
            pos[last] = p;
            if (row4col[j] == -1) sink = j;
            else i = row4col[j];
            SC[j] = 1;
        }
        u[cur] += minVal;
        for (int r = 0; r < nr; ++r)
            if (SR[r] && r != cur) u[r] += minVal - spc[col4row[r]];
        for (int c = 0; c < nc; ++c)
            if (SC[c]) v[c] -= minVal - spc[c];
        int j = sink;
        while (true) {
            const int r = (int)path[j];
            row4col[j] = r;
            std::swap(col4row[r], j);
            if (r == cur) break;
        }
    }
    return 0;
}

// Same solver reading float32 costs straight from the caller's rows (cost = -s, converted to
// double per lane as scipy does, so every reduced cost is bit-identical), with the remaining-set
// as a bit mask, and ONE pass per Dijkstra step: each lane tracks its minimum together with the
// tie key of its holders, which selects the same column as the scalar tie rule without a second
// scan.  The scalar rule picks the last unassigned holder of the minimum in scan order, else the
// first holder; one 32-bit key per column encodes both -- tkey = 2^30 + pos for an unassigned
// column, 2^30 - 1 - pos for an assigned one -- so the rule is "largest key among the holders"
// (one masked max per 8 columns instead of two key tracks).  Keys change with pos (swap-remove:
// one scalar update) and with row4col (only at the augmentation, after the row's search; rebuilt
// with pos at the next row's start).  The float rows hold s (cost = -s); visited rows / columns
// are kept as lists.
//
// The solver is a state machine advanced one Dijkstra step per call (step()), so that one thread
// can interleave two pairs' solves step by step (lsap_solve_f512_x2): a step ends in a serial
// chain -- lane reduction, column selection, row4col lookup -- that the next step's scan depends
// on; the other pair's scan is independent of it and fills the core meanwhile.
constexpr int F512_KU = 1 << 30;   // tie key base of unassigned columns

struct F512Solve {
    int nr = 0, nc = 0, ncp = 0;
    const float* cost = nullptr;
    long ld = 0;
    std::vector<double> u, v, spc;
    std::vector<unsigned char> remb;
    std::vector<int> path, row4col, remaining, pos, tkey, col4row, rows_v, cols_v;
    unsigned char tailm = 0xff;
    int cur = 0, i = 0, num = 0, nrv = 0, ncv = 0;   // nrv / ncv: visited rows / columns this row
    double minVal = 0.0;

    void init(int nr_, int nc_, const float* c, long ld_) {
        nr = nr_; nc = nc_; cost = c; ld = ld_;
        ncp = (nc + 7) & ~7;                               // ncp: read 8 lanes at a time
        u.assign(nr, 0.0); v.assign(ncp, 0.0); spc.assign(ncp, INFINITY);
        remb.assign(ncp / 8, 0xff);
        path.assign(ncp, -1); row4col.assign(ncp, -1); remaining.assign(nc, 0); pos.assign(ncp, 0);
        tkey.assign(ncp, 0);
        col4row.assign(nr, -1);
        rows_v.assign(nr + 1, 0); cols_v.assign(nc + 1, 0);
        tailm = (unsigned char)((nc & 7) ? ((1u << (nc & 7)) - 1) : 0xff);
        cur = 0;
        row_start();
    }
    void row_start() {
        minVal = 0.0;
        i = cur;
        num = nc;
        // locals: the int stores below must not make the compiler re-read members (vectorised)
        const int n = nc, n8 = ncp;
        int* rem = remaining.data();
        int* ps = pos.data();
        int* tk = tkey.data();
        const int* r4c = row4col.data();
        for (int it = 0; it < n; ++it) {
            rem[it] = n - it - 1;
            ps[n - it - 1] = it;
        }
        for (int j = 0; j < n; ++j) tk[j] = r4c[j] == -1 ? F512_KU + ps[j] : F512_KU - 1 - ps[j];
        unsigned char* rb = remb.data();
        for (int q = 0; q < n8 / 8; ++q) rb[q] = 0xff;
        rb[n8 / 8 - 1] = tailm;
        double* sp = spc.data();
        for (int j = 0; j < n8; ++j) sp[j] = INFINITY;
        nrv = ncv = 0;
    }
    // one Dijkstra step of row cur's search: 0 running, 1 solved (col4row final), -1 infeasible
    __attribute__((target("avx512f,avx512dq,avx512vl,avx512bw"), always_inline)) inline int step() {
        const int i0 = i;
        rows_v[nrv++] = i0;
        const float* srow = cost + (long)i0 * ld;
        const unsigned char* rb = remb.data();
        const double* vp = v.data();
        double* sp = spc.data();
        int* pp = path.data();
        const int* kp = tkey.data();
        const int n8 = ncp;
        const __m512d vinf = _mm512_set1_pd(INFINITY);
        const __m512d vmv = _mm512_set1_pd(minVal), vui = _mm512_set1_pd(u[i0]);
        const __m256i vi = _mm256_set1_epi32(i0);
        // one pass: relax the reduced costs and, per lane, track the minimum with the largest
        // tie key among its holders (the scalar loop's tie rule, header above)
        const __m256i m1 = _mm256_set1_epi32(-1);
        __m512d vlow[2] = {vinf, vinf};
        __m256i bk[2] = {m1, m1};
        // full blocks load all 8 floats (removed columns' lanes are masked out of every compare);
        // the tail block past nc loads under the tail mask only
#define FPM_LSA_STEP(jj, a, LOAD)                                                                             \
    {                                                                                                         \
        const int j_ = (jj);                                                                                  \
        const __mmask8 m = rb[j_ >> 3];                                                                       \
        const __m512d c = _mm512_cvtps_pd(LOAD);                                                              \
        const __m512d r = _mm512_sub_pd(_mm512_sub_pd(_mm512_sub_pd(vmv, c), vui), _mm512_loadu_pd(vp + j_)); \
        __m512d sv = _mm512_loadu_pd(sp + j_);                                                                \
        const __mmask8 lt = _mm512_mask_cmp_pd_mask(m, r, sv, _CMP_LT_OQ);                                    \
        sv = _mm512_mask_blend_pd(lt, sv, r);                                                                 \
        _mm512_storeu_pd(sp + j_, sv);                                                                        \
        _mm256_mask_storeu_epi32(pp + j_, lt, vi);                                                            \
        const __mmask8 nl = _mm512_mask_cmp_pd_mask(m, sv, vlow[a], _CMP_LT_OQ);                              \
        const __mmask8 eq = _mm512_mask_cmp_pd_mask(m, sv, vlow[a], _CMP_EQ_OQ);                              \
        const __m256i K = _mm256_loadu_si256((const __m256i*)(kp + j_));                                      \
        vlow[a] = _mm512_mask_blend_pd(nl, vlow[a], sv);                                                      \
        bk[a] = _mm256_mask_max_epi32(_mm256_mask_mov_epi32(bk[a], nl, K), eq, bk[a], K);                     \
    }
        const int nfull = nc & ~7;
        int jj = 0;
        for (; jj + 16 <= nfull; jj += 16) {
            FPM_LSA_STEP(jj, 0, _mm256_loadu_ps(srow + j_))
            FPM_LSA_STEP(jj + 8, 1, _mm256_loadu_ps(srow + j_))
        }
        if (jj < nfull) {
            FPM_LSA_STEP(jj, 0, _mm256_loadu_ps(srow + j_))
            jj += 8;
        }
        if (jj < n8) FPM_LSA_STEP(jj, 1, _mm256_maskz_loadu_ps(tailm, srow + j_))
#undef FPM_LSA_STEP
        // merge the two accumulators lane-wise, then across lanes
        {
            const __mmask8 lo1 = _mm512_cmp_pd_mask(vlow[1], vlow[0], _CMP_LT_OQ);
            const __mmask8 eq1 = _mm512_cmp_pd_mask(vlow[1], vlow[0], _CMP_EQ_OQ);
            vlow[0] = _mm512_mask_blend_pd(lo1, vlow[0], vlow[1]);
            bk[0] = _mm256_mask_max_epi32(_mm256_mask_mov_epi32(bk[0], lo1, bk[1]), eq1, bk[0], bk[1]);
        }
        const double lowest = _mm512_reduce_min_pd(vlow[0]);
        if (lowest == INFINITY) return -1;
        const __mmask8 at = _mm512_cmp_pd_mask(vlow[0], _mm512_set1_pd(lowest), _CMP_EQ_OQ);
        // largest key among the lanes holding the minimum, branch-free (the lane mask is data)
        __m256i kq = _mm256_mask_mov_epi32(m1, at, bk[0]);
        kq = _mm256_max_epi32(kq, _mm256_permute2x128_si256(kq, kq, 1));
        kq = _mm256_max_epi32(kq, _mm256_shuffle_epi32(kq, 0x4e));
        kq = _mm256_max_epi32(kq, _mm256_shuffle_epi32(kq, 0xb1));
        const int kb = _mm256_cvtsi256_si32(kq);
        int* rem = remaining.data();
        int* ps = pos.data();
        const int* r4c = row4col.data();
        const int j = rem[kb >= F512_KU ? kb - F512_KU : F512_KU - 1 - kb];
        minVal = lowest;
        remb[j >> 3] &= (unsigned char)~(1u << (j & 7));
        const int p = ps[j], last = rem[--num];
        rem[p] = last;
        ps[last] = p;
        tkey[last] = r4c[last] == -1 ? F512_KU + p : F512_KU - 1 - p;
        cols_v[ncv++] = j;
        if (r4c[j] != -1) {
            i = r4c[j];
            return 0;
        }
        // sink = j: update the potentials and augment along the path
        const double mv = lowest;
        const int c0 = cur;
        double* uu = u.data();
        double* vv = v.data();
        int* c4r = col4row.data();
        int* r4cw = row4col.data();
        uu[c0] += mv;
        for (int q = 0; q < nrv; ++q) {
            const int r = rows_v[q];
            if (r != c0) uu[r] += mv - sp[c4r[r]];
        }
        for (int q = 0; q < ncv; ++q) {
            const int c = cols_v[q];
            vv[c] -= mv - sp[c];
        }
        int jn = j;
        while (true) {
            const int r = pp[jn];
            r4cw[jn] = r;
            std::swap(c4r[r], jn);
            if (r == c0) break;
        }
        if (++cur == nr) return 1;
        row_start();
        return 0;
    }
};

// one solve to the end: 1 solved, -1 infeasible
__attribute__((target("avx512f,avx512dq,avx512vl,avx512bw"))) int lsap_solve_f512(F512Solve* s) {
    int rc = s->nr > 0 ? 0 : 1;
    while (rc == 0) rc = s->step();
    return rc;
}

// two independent solves, interleaved step by step on this thread
__attribute__((target("avx512f,avx512dq,avx512vl,avx512bw"))) void lsap_solve_f512_x2(F512Solve* s[2], int rc[2]) {
    for (int k = 0; k < 2; ++k) rc[k] = s[k]->nr > 0 ? 0 : 1;
    while (rc[0] == 0 && rc[1] == 0) {
        rc[0] = s[0]->step();
        rc[1] = s[1]->step();
    }
    for (int k = 0; k < 2; ++k)
        while (rc[k] == 0) rc[k] = s[k]->step();
}


// 0 scalar, 1 AVX2, 2 AVX-512 dense scan, 3 AVX-512 float rows + one-pass ties (default where
// available).  FPM_LSA_SCALAR=1 / FPM_LSA_AVX2=1 / FPM_LSA_DENSE512=1 force the older paths.
int lsa_isa() {
#if defined(__x86_64__)
    static int isa = -1;
    if (isa < 0) {
        const char* e = getenv("FPM_LSA_SCALAR");
        const char* a = getenv("FPM_LSA_AVX2");
        const char* d = getenv("FPM_LSA_DENSE512");
        const bool f512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq");
        const bool vlbw = __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512bw");
        if (e && e[0] == '1') isa = 0;
        else if (f512 && !(a && a[0] == '1')) isa = (vlbw && !(d && d[0] == '1')) ? 3 : 2;
        else isa = __builtin_cpu_supports("avx2") ? 1 : 0;
    }
    return isa;
#else
    return 0;
#endif
}


// One pair on the float-row solver: validate s, lay the cost rows out (s's rows, or its
// transpose's when n2 < n1, as scipy transposes tall matrices) and write the assignment back.
struct F512Pair {
    const float* s;
    long ld;
    int n1, n2, n1max;
    int* assign;
    bool tr = false;
    std::vector<float> st;
    F512Solve sv;

    // 1: nothing to solve (empty), -2: NaN / -inf cost, 0: solver initialised
    int prepare() {
        for (int r = 0; r < n1max; ++r) assign[r] = -1;
        if (n1 <= 0 || n2 <= 0) return 1;
        tr = n2 < n1;
        const int nr = tr ? n2 : n1, nc = tr ? n1 : n2;
        for (int i = 0; i < n1; ++i)
            for (int j = 0; j < n2; ++j) {
                const float x = s[(long)i * ld + j];
                if (x != x || x == INFINITY) return -2;     // cost NaN or -inf (scipy raises)
            }
        const float* rows = s;
        long lds = ld;
        if (tr) {
            st.resize((size_t)nr * nc);
            for (int i = 0; i < n1; ++i)
                for (int j = 0; j < n2; ++j) st[(size_t)j * nc + i] = s[(long)i * ld + j];
            rows = st.data();
            lds = nc;
        }
        sv.init(nr, nc, rows, lds);
        return 0;
    }
    void finish() {
        const std::vector<int>& c4r = sv.col4row;
        if (!tr) {
            for (int i = 0; i < sv.nr; ++i) assign[i] = c4r[i];
        } else {
            for (int j = 0; j < sv.nr; ++j) assign[c4r[j]] = j;
        }
    }
};

// Two pairs on one thread with their Dijkstra steps interleaved (ISA path 3 only; see F512Solve).
// rc[k] as lsa_pair's return value.
void lsa_pair_x2(F512Pair* pr[2], int rc[2]) {
    F512Solve* live[2];
    int idx[2], nl = 0;
    for (int k = 0; k < 2; ++k) {
        const int r = pr[k]->prepare();
        rc[k] = r == -2 ? -2 : 0;
        if (r == 0) {
            idx[nl] = k;
            live[nl++] = &pr[k]->sv;
        }
    }
    int src[2] = {1, 1};
    if (nl == 2) {
        lsap_solve_f512_x2(live, src);
    } else if (nl == 1) {
        src[0] = lsap_solve_f512(live[0]);
    }
    for (int q = 0; q < nl; ++q) {
        if (src[q] < 0) rc[idx[q]] = -1;
        else pr[idx[q]]->finish();
    }
}

// one pair: s (ld stride) block [n1 x n2], maximise s  ->  assign[r] = col or -1
int lsa_pair(const float* s, long ld, int n1, int n2, int* assign, int n1max) {
#if defined(__x86_64__)
    if (lsa_isa() == 3) {
        // s's float rows (or its transpose's) are the cost rows; cost = -s inside the scan
        F512Pair p{s, ld, n1, n2, n1max, assign};
        const int r = p.prepare();
        if (r) return r == 1 ? 0 : r;
        if (lsap_solve_f512(&p.sv) < 0) return -1;
        p.finish();
        return 0;
    }
#endif
    for (int r = 0; r < n1max; ++r) assign[r] = -1;
    if (n1 <= 0 || n2 <= 0) return 0;
    const bool tr = n2 < n1;
    const int nr = tr ? n2 : n1, nc = tr ? n1 : n2;
    std::vector<double> cost((size_t)nr * nc);
    for (int i = 0; i < n1; ++i)
        for (int j = 0; j < n2; ++j) {
            const float c = s[(long)i * ld + j] * -1.0f;     // hungarian.py:220 (float32 negation)
            const double d = (double)c;
            if (tr) cost[(size_t)j * nc + i] = d;
            else cost[(size_t)i * nc + j] = d;
        }
    for (size_t k = 0; k < cost.size(); ++k)
        if (cost[k] != cost[k] || cost[k] == -INFINITY) return -2;   // invalid (scipy raises)
    std::vector<int> c4r;
#if defined(__x86_64__)
    const int isa = lsa_isa();
    int rc = isa == 2   ? lsap_solve_dense512(nr, nc, cost.data(), c4r)
             : isa == 1 ? lsap_solve_dense(nr, nc, cost.data(), c4r)
                        : lsap_solve(nr, nc, cost.data(), c4r);
#else
    int rc = lsap_solve(nr, nc, cost.data(), c4r);
#endif
    if (rc) return rc;
    if (!tr) {
        for (int i = 0; i < nr; ++i) assign[i] = c4r[i];
    } else {
        for (int j = 0; j < nr; ++j) assign[c4r[j]] = j;    // rows of the original are columns here
    }
    return 0;
}

// Pairs per worker task: 1 (default) = one pair per task; FPM_LSA_X2=1 -> 2 = two pairs' solves
// interleaved on one thread (lsa_pair_x2, AVX-512 path only).  Interleaving raises one thread's
// throughput ~3 % (EPYC 9575F, n = 256) but halves the workers a batch spreads over, and the
// pipelined forward's tail groups are latency-bound: the 128-pair share line measured 20.0 K pairs/s
// with it vs 20.9 K without (profiles/r05_lsa_host_ab.txt).
int lsa_group() {
    static int g = -1;
    if (g < 0) {
        const char* e = getenv("FPM_LSA_X2");
        g = (e && e[0] == '1') ? 2 : 1;
    }
    return g;
}

// pairs a and b of a batch (b < 0: a only); rc[k] as lsa_pair's return value
void lsa_two(const float* s, long sb, long ld, const int* n1, const int* n2, int n1max, int* assign, int a, int b,
             int rc[2]) {
#if defined(__x86_64__)
    if (b >= 0 && lsa_isa() == 3) {
        F512Pair pa{s + (long)a * sb, ld, n1[a], n2[a], n1max, assign + (long)a * n1max};
        F512Pair pb{s + (long)b * sb, ld, n1[b], n2[b], n1max, assign + (long)b * n1max};
        F512Pair* pr[2] = {&pa, &pb};
        lsa_pair_x2(pr, rc);
        return;
    }
#endif
    rc[0] = lsa_pair(s + (long)a * sb, ld, n1[a], n2[a], assign + (long)a * n1max, n1max);
    rc[1] = b >= 0 ? lsa_pair(s + (long)b * sb, ld, n1[b], n2[b], assign + (long)b * n1max, n1max) : 0;
}

thread_local char g_lsa_err[256];

// Persistent worker pool (created on first use, sized to the largest request seen).
class Pool {
  public:
    void run(int nthreads, int ntasks, const std::function<void(int)>& fn) {
        std::unique_lock<std::mutex> lk(mu_);
        while ((int)workers_.size() < nthreads - 1) {
            const int idx = (int)workers_.size();
            const long g = gen_;     // generation before this run's increment: the worker joins it
            workers_.emplace_back([this, idx, g] { loop(idx, g); });
        }
        fn_ = &fn;
        ntasks_ = ntasks;
        next_.store(0);
        active_ = nthreads - 1;
        done_ = 0;
        ++gen_;
        cv_.notify_all();
        lk.unlock();
        drain();
        lk.lock();
        done_cv_.wait(lk, [this] { return done_ == active_; });
        fn_ = nullptr;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    void drain() {
        while (true) {
            int t = next_.fetch_add(1);
            if (t >= ntasks_) break;
            (*fn_)(t);
        }
    }
    void loop(int idx, long seen) {
        while (true) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            if (stop_) return;
            const bool mine = idx < active_;
            lk.unlock();
            if (!mine) continue;
            drain();
            lk.lock();
            ++done_;
            if (done_ == active_) done_cv_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* fn_ = nullptr;
    std::atomic<int> next_{0};
    int ntasks_ = 0, active_ = 0, done_ = 0;
    long gen_ = 0;
    bool stop_ = false;
};

Pool& pool() {
    static Pool p;
    return p;
}

// Asynchronous batches: a FIFO of jobs served pair by pair by persistent workers, so a batch's
// pairs start as soon as workers free up -- while the previous batch's slowest pairs still run --
// instead of each batch waiting for the whole pool (fpm_lsa_submit / fpm_lsa_wait).
struct LsaJob {
    const float* s;
    long sb, ld;
    const int* n1;
    const int* n2;
    int B, n1max;
    int* assign;
    std::atomic<int> next{0};
    int done = 0;            // guarded by the queue mutex
    int fail = 0;            // first failing pair + 1
    std::chrono::steady_clock::time_point t0, t1;
    bool started = false;
};

class Queue {
  public:
    long submit(std::unique_ptr<LsaJob> job, int nthreads) {
        std::lock_guard<std::mutex> lk(mu_);
        while ((int)workers_.size() < nthreads) workers_.emplace_back([this] { loop(); });
        const long id = ++last_id_;
        LsaJob* j = job.get();
        jobs_[id] = std::move(job);
        if (j->B > 0) fifo_.push_back(j);
        cv_.notify_all();
        return id;
    }
    // 0 / failing pair + 1 when done (seconds: first pair start -> last pair end); -2 while running
    int wait(long id, bool block, double* seconds) {
        std::unique_lock<std::mutex> lk(mu_);
        auto it = jobs_.find(id);
        if (it == jobs_.end()) return -1;
        LsaJob* j = it->second.get();
        if (!block && j->done < j->B) return -2;
        done_cv_.wait(lk, [&] { return j->done >= j->B; });
        const int rc = j->fail;
        if (seconds) *seconds = j->B > 0 ? std::chrono::duration<double>(j->t1 - j->t0).count() : 0.0;
        jobs_.erase(it);
        return rc;
    }
    // Contract: every ticket is waited before its buffers are released (the Python side drains the
    // outstanding tickets of a forward that stops early, ops.lsa_drain).  At exit the workers stop
    // taking pairs once stop_ is set; a pair already running finishes before the join.
    ~Queue() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        while (true) {
            cv_.wait(lk, [&] { return stop_ || !fifo_.empty(); });
            if (stop_) return;
            LsaJob* j = fifo_.front();
            const int b = j->next.fetch_add(1);
            if (b >= j->B) {                 // every pair of the front job is taken
                if (!fifo_.empty() && fifo_.front() == j) fifo_.pop_front();
                continue;
            }
            // a second pair of the same batch when one is left (interleaved with the first)
            int b2 = -1;
            if (lsa_group() == 2 && b + 1 < j->B) b2 = j->next.fetch_add(1);
            if (b2 >= j->B) b2 = -1;
            if (std::max(b, b2) == j->B - 1 && fifo_.front() == j) fifo_.pop_front();
            if (!j->started) {
                j->started = true;
                j->t0 = std::chrono::steady_clock::now();
            }
            lk.unlock();
            int rc[2];
            lsa_two(j->s, j->sb, j->ld, j->n1, j->n2, j->n1max, j->assign, b, b2, rc);
            lk.lock();
            if (rc[0] && (j->fail == 0 || b + 1 < j->fail)) j->fail = b + 1;
            if (rc[1] && (j->fail == 0 || b2 + 1 < j->fail)) j->fail = b2 + 1;
            j->done += b2 >= 0 ? 2 : 1;
            if (j->done == j->B) {
                j->t1 = std::chrono::steady_clock::now();
                done_cv_.notify_all();
            }
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread> workers_;
    std::deque<LsaJob*> fifo_;
    std::map<long, std::unique_ptr<LsaJob>> jobs_;
    long last_id_ = 0;
    bool stop_ = false;
};

Queue& queue() {
    static Queue q;
    return q;
}

}  // namespace

extern "C" {

// s: (B, n1max, n2max) host float32, row stride ld2 (>= n2max) and batch stride sb.
// assign: (B, n1max) int32 output, -1 = unassigned row.  Returns 0, or the lowest failing pair + 1
// (an atomic min over the workers, as the asynchronous queue keeps it: the same pair is named whatever
// the threads' timing or the FPM_LSA_X2 grouping).
int fpm_lsa_batch_host(const float* s, long sb, long ld, const int* n1, const int* n2, int B, int n1max, int* assign,
                       int nthreads) {
    if (B <= 0) return 0;
    const int grp = lsa_group(), ntasks = (B + grp - 1) / grp;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > ntasks) nthreads = ntasks;
    std::atomic<int> fail(0);                     // 0 = none, else lowest failing pair + 1
    std::function<void(int)> work = [&](int t) {
        const int b = t * grp, b2 = grp == 2 && b + 1 < B ? b + 1 : -1;
        int rc[2];
        lsa_two(s, sb, ld, n1, n2, n1max, assign, b, b2, rc);
        for (int k = 0; k < 2; ++k)
            if (rc[k]) {
                const int mine = (k ? b2 : b) + 1;
                int cur = fail.load();
                while ((cur == 0 || mine < cur) && !fail.compare_exchange_weak(cur, mine)) {
                }
            }
    };
    if (nthreads == 1) {
        for (int t = 0; t < ntasks; ++t) work(t);
    } else {
        static std::mutex call_mu;   // one batch at a time through the shared pool
        std::lock_guard<std::mutex> g(call_mu);
        pool().run(nthreads, ntasks, work);
    }
    return fail.load();
}

// Asynchronous form of fpm_lsa_batch_host: queue the batch (pointers must stay valid until
// fpm_lsa_wait) and return a ticket > 0.  Pairs of successive batches are served first-in first-out
// by nthreads persistent workers.
long fpm_lsa_submit(const float* s, long sb, long ld, const int* n1, const int* n2, int B, int n1max, int* assign,
                    int nthreads) {
    std::unique_ptr<LsaJob> j(new LsaJob());
    j->s = s; j->sb = sb; j->ld = ld; j->n1 = n1; j->n2 = n2;
    j->B = B < 0 ? 0 : B; j->n1max = n1max; j->assign = assign;
    return queue().submit(std::move(j), nthreads < 1 ? 1 : nthreads);
}

// block != 0: wait for the ticket's batch; returns 0 or the first failing pair + 1 (like
// fpm_lsa_batch_host) and releases the ticket.  block == 0: -2 while it is still running.  -1: unknown
// ticket.  seconds (optional): the batch's span from its first pair's start to its last pair's end.
int fpm_lsa_wait(long ticket, int block, double* seconds) {
    return queue().wait(ticket, block != 0, seconds);
}

}  // extern "C"
