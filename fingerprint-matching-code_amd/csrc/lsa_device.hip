// On-device linear sum assignment ("on-GPU LAP alternative ... only if
// exact-optimum equivalence is proven"): the same shortest-augmenting-path solver as the host pool
// (csrc/lsa.cpp lsap_solve, Crouse 2016 = scipy's rectangular LSAP behind utils/hungarian.py:8-66),
// restated for one wavefront per pair so that every decision is bit-identical to it:
//   * costs are (double)(-s) from the float32 input, reduced costs ((minVal + c) - u_i) - v_j;
//   * the scan order of the "remaining" columns (initially nc-1 .. 0, swap-remove on selection)
//     is tracked as a position per column; the selected column is the LAST unassigned column
//     holding the minimum if one exists, else the FIRST column holding it (the scalar loop's tie
//     rule), found with one double-min and one int-min wave reduction;
//   * dual updates and the augmenting-path walk are the scalar ones, in the same order.
// Lane l owns columns j = l + 64 k (k < KC), their v / shortest-path cost / path row / scan position
// live in VGPRs; row duals, col4row and the per-augmentation scratch live in LDS.  Each Dijkstra
// step reads one cost row (coalesced 4-B loads), so a pair costs ~(iterations x row latency); all
// pairs of a chunk run concurrently (one wave each), replacing the host pool and the ds_mat D2H.
#include "fpm_common.h"

namespace {

// Wave reductions without LDS round trips: four DPP steps reduce each 16-lane row (quad swaps,
// half-row and row mirrors), then the four row results are read with v_readlane.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i<CTRL>((int)b), hi = dpp_i<CTRL>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double rl_d(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane), hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_min_d(double v) {
    v = fmin(v, dpp_d<0xB1>(v));    // quad_perm [1,0,3,2]
    v = fmin(v, dpp_d<0x4E>(v));    // quad_perm [2,3,0,1]
    v = fmin(v, dpp_d<0x141>(v));   // row_half_mirror
    v = fmin(v, dpp_d<0x140>(v));   // row_mirror
    return fmin(fmin(rl_d(v, 0), rl_d(v, 16)), fmin(rl_d(v, 32), rl_d(v, 48)));
}
__device__ __forceinline__ int wave_min_i(int v) {
    v = min(v, dpp_i<0xB1>(v));
    v = min(v, dpp_i<0x4E>(v));
    v = min(v, dpp_i<0x141>(v));
    v = min(v, dpp_i<0x140>(v));
    return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
               min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

template <int KC>
__global__ __launch_bounds__(64) void lsa_kernel(const float* __restrict__ S, long sb, long ld, const int* __restrict__ n1v,
                                                 const int* __restrict__ n2v, int n1max, int nmax_all,
                                                 int* __restrict__ assign, int* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int b = blockIdx.x, lane = threadIdx.x;
    const int n1 = n1v[b], n2 = n2v[b];
    int* as = assign + (long)b * n1max;
    for (int r = lane; r < n1max; r += 64) as[r] = -1;
    if (lane == 0) status[b] = 0;
    if (n1 <= 0 || n2 <= 0) return;
    const bool tr = n2 < n1;
    const int nr = tr ? n2 : n1, nc = tr ? n1 : n2;
    const float* sp = S + (long)b * sb;
    const long rstride = tr ? 1 : ld, cstride = tr ? ld : 1;   // cost(i, j) = -s at sp[i*rstride + j*cstride]

    // LDS: u[nmax_all] double, spc[nmax_all] double, col4row, pathL, row4col [nmax_all] int, SR bytes
    double* u = (double*)smem;
    double* spcL = u + nmax_all;
    int* col4row = (int*)(spcL + nmax_all);
    int* pathL = col4row + nmax_all;
    int* row4col = pathL + nmax_all;
    unsigned char* SR = (unsigned char*)(row4col + nmax_all);
    __shared__ int s_bad;

    // scipy raises on NaN / -inf costs (host twin returns -2): s NaN or +inf
    if (lane == 0) s_bad = 0;
    for (int r = lane; r < nr; r += 64) {
        u[r] = 0.0;
        col4row[r] = -1;
    }
    for (int j = lane; j < nc; j += 64) row4col[j] = -1;
    __syncthreads();
    for (long t = lane; t < (long)n1 * n2; t += 64) {
        const int i = (int)(t / n2), j = (int)(t - (long)i * n2);
        const float x = sp[(long)i * ld + j];
        if (x != x || x == INFINITY) s_bad = 1;
    }
    __syncthreads();
    if (s_bad) {
        if (lane == 0) status[b] = 2;
        return;
    }

    double v[KC], rs[KC];
    int pos[KC], path[KC], r4c[KC];   // r4c: row4col of the lane's columns (mirrors LDS row4col)
#pragma unroll
    for (int k = 0; k < KC; ++k) {
        v[k] = 0.0;
        r4c[k] = -1;
    }
    for (int cur = 0; cur < nr; ++cur) {
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int j = lane + 64 * k;
            pos[k] = j < nc ? nc - 1 - j : -1;
            rs[k] = INFINITY;
            path[k] = -1;
        }
        for (int r = lane; r < nr; r += 64) SR[r] = 0;
        __syncthreads();
        double minVal = 0.0;
        int i = cur, num = nc, sink = -1;
        while (sink == -1) {
            if (lane == 0) SR[i] = 1;
            const double ui = u[i];
            const float* row = sp + (long)i * rstride;
            float cf[KC];
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const int j = lane + 64 * k;
                cf[k] = pos[k] >= 0 ? row[(long)j * cstride] : 0.f;
            }
            double lo = INFINITY;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                if (pos[k] >= 0) {
                    const double c = (double)(cf[k] * -1.0f);
                    const double r = ((minVal + c) - ui) - v[k];
                    if (r < rs[k]) {
                        rs[k] = r;
                        path[k] = i;
                    }
                    lo = fmin(lo, rs[k]);
                }
            }
            const double lowest = wave_min_d(lo);
            if (!(lowest < INFINITY)) {
                if (lane == 0) status[b] = 1;   // infeasible
                return;
            }
            // tie rule key: unassigned columns first, by descending position; then by ascending position
            int key = 0x7fffffff;
#pragma unroll
            for (int k = 0; k < KC; ++k)
                if (pos[k] >= 0 && rs[k] == lowest) key = min(key, r4c[k] >= 0 ? 4096 + pos[k] : 4095 - pos[k]);
            key = wave_min_i(key);
            const int p = key >= 4096 ? key - 4096 : 4095 - key;
            int jsel = -1, rsel = -1;
#pragma unroll
            for (int k = 0; k < KC; ++k)
                if (pos[k] == p) {
                    jsel = lane + 64 * k;
                    rsel = r4c[k];
                }
            const unsigned long long own = __ballot(jsel >= 0);
            const int owner = __builtin_amdgcn_readfirstlane(__ffsll((long long)own) - 1);
            const int j = __builtin_amdgcn_readlane(jsel, owner);
            minVal = lowest;
            const int rj = __builtin_amdgcn_readlane(rsel, owner);
            if (rj == -1) sink = j;
            else i = rj;
            // swap-remove position p: the column at position num-1 moves to p, j leaves the scan
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                if (pos[k] == num - 1) pos[k] = p;
                if (lane + 64 * k == j) pos[k] = -2;    // -2: scanned (SC) this augmentation
            }
            --num;
        }
        // dual updates (scalar order: u[cur], SR rows, SC columns), then the path walk
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int j = lane + 64 * k;
            if (j < nc) {
                spcL[j] = rs[k];
                pathL[j] = path[k];
            }
        }
        __syncthreads();
        for (int r = lane; r < nr; r += 64)
            if (SR[r] && r != cur) u[r] += minVal - spcL[col4row[r]];
        if (lane == 0) u[cur] += minVal;
#pragma unroll
        for (int k = 0; k < KC; ++k)
            if (pos[k] == -2) v[k] -= minVal - rs[k];
        __syncthreads();
        if (lane == 0) {
            int j = sink;
            while (true) {
                const int r = pathL[j];
                row4col[j] = r;
                const int t = col4row[r];
                col4row[r] = j;
                j = t;
                if (r == cur) break;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int j = lane + 64 * k;
            r4c[k] = j < nc ? row4col[j] : -1;
        }
    }
    if (!tr) {
        for (int r = lane; r < nr; r += 64) as[r] = col4row[r];
    } else {
        for (int r = lane; r < nr; r += 64) as[col4row[r]] = r;
    }
}

}  // namespace

// s: (B, n1max, n2max)-strided device float32 (row stride ld, batch stride sb); maximise s per pair
// over its n1[b] x n2[b] block.  assign (B, n1max) int32: column of each row or -1.  status (B)
// int32: 0 ok, 1 infeasible, 2 NaN / -inf cost (scipy raises).  n1max, n2max <= 1024.
extern "C" int fpm_lsa_batch_device(const float* s, long sb, long ld, const int* n1, const int* n2, int B, int n1max,
                                    int n2max, int* assign, int* status, void* stream) {
    FPM_CHECK_ARG(B >= 0 && n1max >= 0 && n2max >= 0, "lsa_device: bad sizes");
    FPM_CHECK_ARG(n1max <= 1024 && n2max <= 1024, "lsa_device: n1max/n2max > 1024 (got %d, %d)", n1max, n2max);
    FPM_CHECK_ARG(ld >= n2max && sb >= (long)n1max * ld, "lsa_device: bad strides");
    if (B == 0) return 0;
    const int nall = n1max > n2max ? n1max : n2max;
    const int KC = (nall + 63) / 64;
    const size_t sh = (size_t)nall * (2 * sizeof(double) + 3 * sizeof(int) + 1);
    hipStream_t st = (hipStream_t)stream;
#define FPM_LSA(K)                                                                                            \
    hipLaunchKernelGGL((lsa_kernel<K>), dim3(B), dim3(64), sh, st, s, sb, ld, n1, n2, n1max, nall, assign, status)
    if (KC <= 1) FPM_LSA(1);
    else if (KC <= 2) FPM_LSA(2);
    else if (KC <= 4) FPM_LSA(4);
    else if (KC <= 8) FPM_LSA(8);
    else FPM_LSA(16);
#undef FPM_LSA
    return fpm::check_launch("fpm_lsa_batch_device");
}
