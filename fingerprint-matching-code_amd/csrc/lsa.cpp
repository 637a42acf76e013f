// Host-side linear sum assignment for utils/hungarian.py:8-66 (scipy.optimize.linear_sum_assignment
// on -s), batched over pairs with a pool of std::threads.
//
// Algorithm: shortest augmenting path with dual potentials (Crouse 2016), the method behind
// scipy >= 1.4's rectangular LSAP solver (scipy 1.10.1 pinned at environment.yml:229).  The
// column scan order (remaining columns filled in reverse), the tie rule (prefer an unassigned
// column among equal reduced costs) and the transpose of tall matrices follow that published
// method so that, on inputs with ties, the same optimum is returned.  Costs are evaluated in
// double from the float32 input (-s), as scipy converts its input to float64.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
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

// one pair: s (ld stride) block [n1 x n2], maximise s  ->  assign[r] = col or -1
int lsa_pair(const float* s, long ld, int n1, int n2, int* assign, int n1max) {
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
    int rc = lsap_solve(nr, nc, cost.data(), c4r);
    if (rc) return rc;
    if (!tr) {
        for (int i = 0; i < nr; ++i) assign[i] = c4r[i];
    } else {
        for (int j = 0; j < nr; ++j) assign[c4r[j]] = j;    // rows of the original are columns here
    }
    return 0;
}

thread_local char g_lsa_err[256];

}  // namespace

extern "C" {

// s: (B, n1max, n2max) host float32, row stride ld2 (>= n2max) and batch stride sb.
// assign: (B, n1max) int32 output, -1 = unassigned row.  Returns 0, or the first failing pair+1.
int fpm_lsa_batch_host(const float* s, long sb, long ld, const int* n1, const int* n2, int B, int n1max, int* assign,
                       int nthreads) {
    if (B <= 0) return 0;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > B) nthreads = B;
    std::atomic<int> next(0), fail(0);
    auto work = [&]() {
        while (true) {
            int b = next.fetch_add(1);
            if (b >= B) break;
            int rc = lsa_pair(s + (long)b * sb, ld, n1[b], n2[b], assign + (long)b * n1max, n1max);
            if (rc) {
                int expect = 0;
                fail.compare_exchange_strong(expect, b + 1);
            }
        }
    };
    if (nthreads == 1) {
        work();
    } else {
        std::vector<std::thread> th;
        th.reserve(nthreads);
        for (int t = 0; t < nthreads; ++t) th.emplace_back(work);
        for (auto& t : th) t.join();
    }
    return fail.load();
}

}  // extern "C"
