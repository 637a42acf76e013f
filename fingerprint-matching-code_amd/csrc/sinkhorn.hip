// Log-domain Sinkhorn (pygmtools 0.5.3 ``sinkhorn`` semantics, called at
// reference src/model/sinkhorn.py:87 and src/model/gnn.py:221) — one workgroup per pair, the
// whole n1max x n2max block resident in VGPRs (1024 threads x ER*EC values).
//
// Dual-potential form: L = S/tau - u_row - v_col.  A row step sets u = lse_cols(S/tau - v), a
// column step v = lse_rows(S/tau - u); this is the reference's alternating
// ``L -= logsumexp(L, dim)`` with the running sums kept as potentials, so S is read once and the
// only per-iteration state is u, v.  Semantics kept: row step first, per-pair valid block
// [:n1, :n2], n1 > n2 handled on the transpose, dummy rows (value -100 in log space) when
// dummy_row and rows < cols, output exp(L) on the block and 0 in the padding.
// Arithmetic runs in log2 units (L2 = L log2 e): every exp/log is one native v_exp_f32 / v_log_f32.
#include "fpm_common.h"
#include <cstdlib>
#include <type_traits>

namespace {

struct SinkArgs {
    const float* in;
    long in_sb, in_si, in_sj;
    float* out;
    long out_sb, out_si, out_sj;
    const int* n1;
    const int* n2;
    int n1max, n2max;
    int iters;
    float tau;
    int dummy_row;
    int contig_j;  // 1: j (column) is the unit-stride dimension of in/out
    int fast;      // shifted single-pass lse after the first step (sinkhorn_reg_kernel)
    int rw;        // streaming kernel: rows per wave in the row step's fast path (> 1: multi-row form)
    // streaming kernel, pairs split over `split` workgroups along a (1 = one workgroup per pair):
    // B pairs, per-pair arrival counters (zeroed before the launch), exchange slots of xslot floats
    int B, split;
    int xacq;      // 1: agent acquire fence after each exchange poll (default 0: sc1 loads, no fence)
    int* xcnt;
    float* xbuf;
    long xslot;
    // backward (sinkhorn_reg_kernel<.., true>): dP view, dS out (contiguous B x n1max x n2max),
    // potential history (B x iters x H floats; slot H - 1: the dummy rows' potential)
    const float* dp;
    long dp_sb, dp_si, dp_sj;
    float* ds;
    float* hist;
    float* ds_tile;   // B x (1024 ER EC) scaled input tiles (replay -> sweep)
    int H;
};

__device__ __forceinline__ void lse_combine(float& m, float& s, float mo, float so) {
    float mn = fmaxf(m, mo);
    if (mn == -INFINITY) { m = mn; s = 0.f; return; }
    s = s * fpm::fast_exp2(m - mn) + so * fpm::fast_exp2(mo - mn);
    m = mn;
}

// Reductions over the 32 lanes sharing tr, on the VALU: DPP quad_perm xor 1 / xor 2, then the
// half-row / row mirrors (after the quad steps every lane of a quad holds the same value, so a
// mirror pairs whole quads / half-rows like an xor 4 / xor 8), then v_permlane16_swap for xor 16.
// Every lane of the 32 ends with the bit-identical result (each step adds the same two operands).
// (ds_bpermute shuffles, one LDS round trip per level, left these kernels latency-bound.)
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane32_max(float v) {
    v = fmaxf(v, dppf<0xB1>(v));
    v = fmaxf(v, dppf<0x4E>(v));
    v = fmaxf(v, dppf<0x141>(v));
    v = fmaxf(v, dppf<0x140>(v));
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    return fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}
__device__ __forceinline__ float lane32_sum(float v) {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x141>(v);
    v += dppf<0x140>(v);
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float(r[0]) + __int_as_float(r[1]);
}
// an int the compiler cannot see through (keeps per-thread coordinates from being hoisted and held
// live across the step loop)
__device__ __forceinline__ int opaque_i(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// value of lane ^ 32 (v_permlane32_swap: the two wave halves exchange)
__device__ __forceinline__ float xor32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// BWD = true: the training backward (reference gradient of pygm.sinkhorn through autograd):
// the same forward steps replayed with every step's changed potentials kept in a.hist, then the
// vector-Jacobian product walked in reverse with the gradient tile dL in registers (the input
// block is re-read per step from L2 instead of held: M and dL together exceed the 128-register
// budget of 1024-thread workgroups).  For a step L' = L - lse(L) along one axis,
// dL = dL' - exp(L') * sum(dL') along that axis; the nd identical dummy rows carry one gradient
// row dLd; dS = dL_0 / tau.  Reductions are fixed-order (deterministic).
template <int ER, int EC, bool BWD = false>
__global__ __launch_bounds__(1024) void sinkhorn_reg_kernel(SinkArgs a) {
    constexpr int NCOL = 32 * EC;
    __shared__ float red_m[16][NCOL];
    __shared__ float red_s[16][NCOL];
    __shared__ float fin[NCOL];
    __shared__ float blk_m[16], blk_s[16];
    __shared__ int redo_flag;

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int tr = tid >> 5, tc = tid & 31, wv = tid >> 6;
    const int n1b = a.n1[b], n2b = a.n2[b];
    const bool transposed = n1b > n2b;
    const int R = transposed ? n2b : n1b;   // algorithmic rows
    const int C = transposed ? n1b : n2b;   // algorithmic cols
    const int nd = (a.dummy_row && C > R) ? (C - R) : 0;
    const float lognd = nd > 0 ? fpm::fast_log2((float)nd) : 0.f;
    // physical dims: pc (lanes) = unit-stride dim
    const int limPR = a.contig_j ? n1b : n2b;
    const int limPC = a.contig_j ? n2b : n1b;
    const int boxPR = a.contig_j ? a.n1max : a.n2max;
    const int boxPC = a.contig_j ? a.n2max : a.n1max;
    // u (row potential) lives on the pr side iff the algorithmic row dim is the pr dim
    const bool u_on_R = (a.contig_j != 0) == (!transposed);

    const float* in = a.in + (long)b * a.in_sb;
    const int ispr = (int)(a.contig_j ? a.in_si : a.in_sj);
    const int ispc = (int)(a.contig_j ? a.in_sj : a.in_si);

    float M[ER][EC];
    float pR[ER], pC[EC];
    // S / tau in log2 units as ONE multiply by LOG2E / tau, exactly the L-form forward's load
    // (sinkhorn_lform_kernel): the training backward replays the forward that actually ran
    const float vscale = fpm::LOG2E_F / a.tau;
#pragma unroll
    for (int e = 0; e < ER; ++e) {
        pR[e] = 0.f;
        const int pr = tr + 32 * e;
#pragma unroll
        for (int f = 0; f < EC; ++f) {
            const int pc = tc + 32 * f;
            float v = -INFINITY;
            // 32-bit in-pair offsets (a pair's block is < 2^31 elements): 64-bit address math for
            // the 64 loads held the register tile hostage (spills in the step loop)
            if (pr < limPR && pc < limPC) v = in[pr * ispr + pc * ispc] * vscale;
            M[e][f] = v;
        }
    }
#pragma unroll
    for (int f = 0; f < EC; ++f) pC[f] = 0.f;

    float ud = 0.f;  // potential of the (identical) dummy rows
    const float DUMMY = -100.f * fpm::LOG2E_F;   // the dummy rows' log value, in log2 units

    // Shifted single-pass lse (fast = true, every step after the first): after a normalisation
    // along one axis every entry is <= 0 in log space, so the other axis' lse can be shifted by its
    // own previous potential instead of a max pass -- one exp per entry, no max reduction.  A sum
    // outside [2^-30, 2^30] (unnormalised input, extreme lines) falls back to the max-shifted form.
    auto ok_s = [](float x) { return x >= 0x1p-30f && x <= 0x1p30f; };
    // potR[e] = lse_f(M - pC) (+ dummy term)
    auto update_R = [&](bool add_dummy, bool fast) {
        if (fast) {
            bool bad = false;
            // all ER rows' sums first, then their reductions: ER independent DPP chains in flight.
            // M - (pC + sh), not (M - pC) - sh: the latter is CSE'd with the max-shifted path's
            // M - pC, which then stays live as a second 64-value tile (VGPR spills)
            float s[ER];
#pragma unroll
            for (int e = 0; e < ER; ++e) {
                const float sh = pR[e];
                float t = 0.f;
#pragma unroll
                for (int f = 0; f < EC; ++f) t += fpm::fast_exp2(M[e][f] - (pC[f] + sh));
                s[e] = t;
            }
#pragma unroll
            for (int e = 0; e < ER; ++e) s[e] = lane32_sum(s[e]);
#pragma unroll
            for (int e = 0; e < ER; ++e) {
                float t = s[e];
                if (add_dummy) t += (float)nd * fpm::fast_exp2(DUMMY - ud - pR[e]);
                s[e] = t;
                bad |= !ok_s(t);
            }
            // any row of the wave out of range: the whole wave redoes the step max-shifted (rare;
            // keeps one path live at a time -- per-row fallbacks spilled the register tile)
            if (__ballot(bad) == 0ull) {
#pragma unroll
                for (int e = 0; e < ER; ++e) pR[e] += fpm::fast_log2(s[e]);
                return;
            }
        }
#pragma unroll
        for (int e = 0; e < ER; ++e) {
            float m = -INFINITY;
#pragma unroll
            for (int f = 0; f < EC; ++f) m = fmaxf(m, M[e][f] - pC[f]);
            m = lane32_max(m);
            float dv = DUMMY - ud;
            if (add_dummy) m = fmaxf(m, dv);
            float s = 0.f;
            if (m != -INFINITY) {
#pragma unroll
                for (int f = 0; f < EC; ++f) s += fpm::fast_exp2(M[e][f] - (pC[f] + m));
            }
            s = lane32_sum(s);
            if (add_dummy && m != -INFINITY) s += (float)nd * fpm::fast_exp2(dv - m);
            pR[e] = (m == -INFINITY) ? 0.f : m + fpm::fast_log2(s);
        }
    };
    // potC[f] = lse_e(M - pR) (+ dummy term): across the 32 thread-rows via LDS
    auto update_C = [&](bool add_dummy, bool fast) {
        if (fast) {
            float cs[EC];
#pragma unroll
            for (int f = 0; f < EC; ++f) {
                float s = 0.f;
#pragma unroll
                for (int e = 0; e < ER; ++e) s += fpm::fast_exp2(M[e][f] - (pR[e] + pC[f]));
                cs[f] = s;
            }
#pragma unroll
            for (int f = 0; f < EC; ++f) {
                const float s = cs[f] + xor32(cs[f]);
                if ((tid & 63) < 32) red_s[wv][tc + 32 * f] = s;
                if (tr == 0) fin[tc + 32 * f] = pC[f];            // the old potentials (shifts)
            }
            __syncthreads();
            if (tid < NCOL) {
                float s = red_s[0][tid];
                for (int w = 1; w < 16; ++w) s += red_s[w][tid];
                const float sh = fin[tid];
                if (add_dummy) s += (float)nd * fpm::fast_exp2(DUMMY - ud - sh);
                // columns past the valid block carry no entries (only the dummy term, as below)
                if (tid >= limPC) red_m[0][tid] = add_dummy ? (DUMMY - ud) + lognd : 0.f;
                else if (ok_s(s)) red_m[0][tid] = sh + fpm::fast_log2(s);
                else redo_flag = 1;                               // any failure: redo the step
            }
            __syncthreads();
            const bool redo = redo_flag != 0;
            if (!redo) {
#pragma unroll
                for (int f = 0; f < EC; ++f) pC[f] = red_m[0][tc + 32 * f];
                return;
            }
        }
#pragma unroll
        for (int f = 0; f < EC; ++f) {
            float m = -INFINITY;
#pragma unroll
            for (int e = 0; e < ER; ++e) m = fmaxf(m, M[e][f] - pR[e]);
            float s = 0.f;
            if (m != -INFINITY) {
#pragma unroll
                for (int e = 0; e < ER; ++e) s += fpm::fast_exp2(M[e][f] - (pR[e] + m));
            }
            float mo = xor32(m), so = xor32(s);
            lse_combine(m, s, mo, so);
            if ((tid & 63) < 32) {
                red_m[wv][tc + 32 * f] = m;
                red_s[wv][tc + 32 * f] = s;
            }
        }
        __syncthreads();
        if (tid < NCOL) {
            float m = red_m[0][tid], s = red_s[0][tid];
            for (int w = 1; w < 16; ++w) lse_combine(m, s, red_m[w][tid], red_s[w][tid]);
            if (add_dummy) lse_combine(m, s, DUMMY - ud, (float)nd);
            fin[tid] = (m == -INFINITY) ? 0.f : m + fpm::fast_log2(s);
        }
        __syncthreads();
#pragma unroll
        for (int f = 0; f < EC; ++f) pC[f] = fin[tc + 32 * f];
        if (fast) {   // reset the redo flag (read by every thread above, before this barrier)
            if (tid == 0) redo_flag = 0;
            __syncthreads();
        }
    };
    // ud = lse over valid algorithmic columns of (-100 - v)
    auto update_dummy = [&]() {
        float m = -INFINITY, s = 0.f;
        if (u_on_R) {  // v on the pc side
#pragma unroll
            for (int f = 0; f < EC; ++f)
                if (tc + 32 * f < limPC) m = fmaxf(m, DUMMY - pC[f]);
            m = lane32_max(m);
#pragma unroll
            for (int f = 0; f < EC; ++f)
                if (tc + 32 * f < limPC) s += fpm::fast_exp2(DUMMY - pC[f] - m);
            s = lane32_sum(s);
            ud = m + fpm::fast_log2(s);
        } else {       // v on the pr side: block reduction over threads with tc == 0
            if (tc == 0) {
#pragma unroll
                for (int e = 0; e < ER; ++e)
                    if (tr + 32 * e < limPR) m = fmaxf(m, DUMMY - pR[e]);
#pragma unroll
                for (int e = 0; e < ER; ++e)
                    if (tr + 32 * e < limPR) s += fpm::fast_exp2(DUMMY - pR[e] - m);
            }
            float mo = xor32(m), so = xor32(s);
            lse_combine(m, s, mo, so);
            if ((tid & 63) == 0) { blk_m[wv] = m; blk_s[wv] = s; }
            __syncthreads();
            m = blk_m[0]; s = blk_s[0];
            for (int w = 1; w < 16; ++w) lse_combine(m, s, blk_m[w], blk_s[w]);
            ud = m + fpm::fast_log2(s);
            __syncthreads();
        }
    };

    if (tid == 0) redo_flag = 0;
    __syncthreads();
    float* hist = BWD ? a.hist + (long)b * a.iters * a.H : nullptr;
    // the physical side a step updates: R iff (row step) == u_on_R
    auto save = [&](int it, bool Rside) {
        float* h = hist + (long)it * a.H;
        if (Rside) {
            if (tc == 0) {
#pragma unroll
                for (int e = 0; e < ER; ++e)
                    if (tr + 32 * e < boxPR) h[tr + 32 * e] = pR[e];
            }
        } else if (tr == 0) {
#pragma unroll
            for (int f = 0; f < EC; ++f)
                if (tc + 32 * f < boxPC) h[tc + 32 * f] = pC[f];
        }
        if (tid == 0) h[a.H - 1] = ud;
    };
    for (int it = 0; it < a.iters; ++it) {
        const bool fast = it > 0 && a.fast;
        if ((it & 1) == 0) {           // row normalisation: update u
            if (u_on_R) update_R(false, fast); else update_C(false, fast);
            if (nd > 0) update_dummy();
        } else {                       // column normalisation: update v
            if (u_on_R) update_C(nd > 0, fast); else update_R(nd > 0, fast);
        }
        if constexpr (BWD) save(it, ((it & 1) == 0) == u_on_R);
    }
    (void)lognd;
    if constexpr (BWD) {
        // replay only: keep the scaled input tile (-inf padding included) for the sweep kernel,
        // [e * EC + f][thread] -- coalesced, and re-read there without bounds checks
        float* tile = a.ds_tile + (long)b * (1024 * ER * EC) + tid;
#pragma unroll
        for (int e = 0; e < ER; ++e)
#pragma unroll
            for (int f = 0; f < EC; ++f) tile[(e * EC + f) * 1024] = M[e][f];
        return;                             // the reverse steps: sinkhorn_bwd_sweep_kernel
    }

    float* out = a.out + (long)b * a.out_sb;
    const int opr = (int)(a.contig_j ? a.out_si : a.out_sj);
    const int opc = (int)(a.contig_j ? a.out_sj : a.out_si);
#pragma unroll
    for (int e = 0; e < ER; ++e) {
        const int pr = tr + 32 * e;
        if (pr >= boxPR) continue;
#pragma unroll
        for (int f = 0; f < EC; ++f) {
            const int pc = tc + 32 * f;
            if (pc >= boxPC) continue;
            float v = 0.f;
            if (pr < limPR && pc < limPC) v = fpm::fast_exp2(M[e][f] - pR[e] - pC[f]);
            out[pr * opr + pc * opc] = v;
        }
    }
}

// Reverse sweep of the Sinkhorn backward (after sinkhorn_reg_kernel<ER, EC, true> replayed the
// forward into a.hist): its own kernel so the gradient tile dL gets the register budget the
// forward's tile M had (both phases in one kernel spilled ~300 VGPRs).
template <int ER, int EC>
__global__ __launch_bounds__(1024) void sinkhorn_bwd_sweep_kernel(SinkArgs a) {
    constexpr int NCOL = 32 * EC;
    __shared__ float red_s[16][NCOL];
    __shared__ float fin[NCOL];
    __shared__ float blk_s[16];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int tr = tid >> 5, tc = tid & 31, wv = tid >> 6;
    const int n1b = a.n1[b], n2b = a.n2[b];
    const bool transposed = n1b > n2b;
    const int R = transposed ? n2b : n1b;
    const int C = transposed ? n1b : n2b;
    const int nd = (a.dummy_row && C > R) ? (C - R) : 0;
    const int limPR = a.contig_j ? n1b : n2b;
    const int limPC = a.contig_j ? n2b : n1b;
    const int boxPR = a.contig_j ? a.n1max : a.n2max;
    const int boxPC = a.contig_j ? a.n2max : a.n1max;
    const bool u_on_R = (a.contig_j != 0) == (!transposed);
    const float* in = a.in + (long)b * a.in_sb;
    const int ispr = (int)(a.contig_j ? a.in_si : a.in_sj);
    const int ispc = (int)(a.contig_j ? a.in_sj : a.in_si);
    const float DUMMY = -100.f * fpm::LOG2E_F;
    const float* hist = a.hist + (long)b * a.iters * a.H;
    // potentials after the last step: its side from hist[T-1], the other side from hist[T-2]
    float pR[ER], pC[EC], ud = 0.f;
    {
        const int T = a.iters;
        const bool lastR = T > 0 && (((T - 1) & 1) == 0) == u_on_R;
        const int sR = lastR ? T - 1 : T - 2, sC = lastR ? T - 2 : T - 1;   // slot per side (< 0: none)
        const float* hR = hist + (long)(sR > 0 ? sR : 0) * a.H;
        const float* hC = hist + (long)(sC > 0 ? sC : 0) * a.H;
#pragma unroll
        for (int e = 0; e < ER; ++e) {
            const int r = tr + 32 * e;
            const float v = T > 0 ? hR[min(r, a.H - 2)] : 0.f;
            pR[e] = (sR >= 0 && r < boxPR) ? v : 0.f;
        }
#pragma unroll
        for (int f = 0; f < EC; ++f) {
            const int c = tc + 32 * f;
            const float v = T > 0 ? hC[min(c, a.H - 2)] : 0.f;
            pC[f] = (sC >= 0 && c < boxPC) ? v : 0.f;
        }
        if (T > 0) ud = hist[(long)(T - 1) * a.H + a.H - 1];
    }
    // the scaled input tile the replay kept, re-read per step (unconditional coalesced loads; -inf
    // in the padding).  z is an opaque 0 renewed every step so the loads stay inside the step loop
    // (bounds-checked re-reads of the input, or hoisted loads, spilled ~250 VGPRs)
    int z = 0;
    const float* tileM = a.ds_tile + (long)b * (1024 * ER * EC) + tid;
    auto Mv = [&](int e, int f) { return tileM[(e * EC + f) * 1024 + z]; };
    (void)in; (void)ispr; (void)ispc;
    auto validR = [&](int e) { return tr + 32 * e < limPR; };
    auto validC = [&](int f) { return tc + 32 * f < limPC; };
    // dL_T = dP o P_T on the real rows (dummy rows get no direct gradient)
    const float* dpb = a.dp + (long)b * a.dp_sb;
    const int dpr = (int)(a.contig_j ? a.dp_si : a.dp_sj), dpc = (int)(a.contig_j ? a.dp_sj : a.dp_si);
    // dL: rows e < EREG in registers, the rest in LDS ([e - EREG][f][thread], conflict-free)
    constexpr int EREG = ER >= 8 ? ER / 2 : ER;
    extern __shared__ float dLs[];
    float dLr[EREG][EC], dLd[ER];
    auto DL = [&](int e, int f) -> float& {
        return e < EREG ? dLr[e < EREG ? e : 0][f] : dLs[((e - EREG) * EC + f) * 1024 + tid];
    };
#pragma unroll
    for (int e = 0; e < ER; ++e) {
        dLd[e] = 0.f;
        const int pr = tr + 32 * e;
#pragma unroll
        for (int f = 0; f < EC; ++f) {
            const int pc = tc + 32 * f;
            float g = 0.f;
            if (pr < limPR && pc < limPC) g = dpb[pr * dpr + pc * dpc] * fpm::fast_exp2(Mv(e, f) - pR[e] - pC[f]);
            DL(e, f) = g;
        }
    }
        for (int t = a.iters - 1; t >= 0; --t) {
            z = 0;
            asm volatile("" : "+v"(z));
            const bool algrow = (t & 1) == 0;
            const bool Rside = algrow == u_on_R;          // physical side this step normalised
            const bool dsum = !algrow && nd > 0;           // column step: dummy rows in the sums
            if (Rside) {
                float sr[ER];
#pragma unroll
                for (int e = 0; e < ER; ++e) {
                    float t2 = 0.f;
#pragma unroll
                    for (int f = 0; f < EC; ++f) t2 += DL(e, f);
                    sr[e] = t2;
                }
#pragma unroll
                for (int e = 0; e < ER; ++e) sr[e] = lane32_sum(sr[e]);
#pragma unroll
                for (int e = 0; e < ER; ++e) {
                    if (dsum) sr[e] = fmaf((float)nd, dLd[e], sr[e]);
#pragma unroll
                    for (int f = 0; f < EC; ++f) DL(e, f) -= fpm::fast_exp2(Mv(e, f) - pR[e] - pC[f]) * sr[e];
                    if (dsum && validR(e)) dLd[e] -= fpm::fast_exp2(DUMMY - ud - pR[e]) * sr[e];
                    __builtin_amdgcn_sched_barrier(0);     // one row's 8 loads in flight at a time
                }
            } else {
                float cs[EC];
#pragma unroll
                for (int f = 0; f < EC; ++f) {
                    float t2 = 0.f;
#pragma unroll
                    for (int e = 0; e < ER; ++e) t2 += DL(e, f);
                    cs[f] = t2;
                }
#pragma unroll
                for (int f = 0; f < EC; ++f) {
                    const float v = cs[f] + xor32(cs[f]);
                    if ((tid & 63) < 32) red_s[wv][tc + 32 * f] = v;
                }
                __syncthreads();
                if (tid < NCOL) {
                    float v = red_s[0][tid];
                    for (int w = 1; w < 16; ++w) v += red_s[w][tid];
                    fin[tid] = v;
                }
                __syncthreads();
#pragma unroll
                for (int f = 0; f < EC; ++f) {
                    float sc = fin[tc + 32 * f];
                    if (dsum) sc = fmaf((float)nd, dLd[f], sc);
#pragma unroll
                    for (int e = 0; e < ER; ++e) DL(e, f) -= fpm::fast_exp2(Mv(e, f) - pR[e] - pC[f]) * sc;
                    if (dsum && validC(f)) dLd[f] -= fpm::fast_exp2(DUMMY - ud - pC[f]) * sc;
                    __builtin_amdgcn_sched_barrier(0);
                }
                __syncthreads();                            // fin / red_s reused
            }
            if (algrow && nd > 0) {
                // the dummy rows' own row step: their sum over the valid algorithmic columns
                if (u_on_R) {
                    float sd = 0.f;
#pragma unroll
                    for (int f = 0; f < EC; ++f)
                        if (validC(f)) sd += dLd[f];
                    sd = lane32_sum(sd);
#pragma unroll
                    for (int f = 0; f < EC; ++f)
                        if (validC(f)) dLd[f] -= fpm::fast_exp2(DUMMY - ud - pC[f]) * sd;
                } else {
                    float sd = 0.f;
                    if (tc == 0) {
#pragma unroll
                        for (int e = 0; e < ER; ++e)
                            if (validR(e)) sd += dLd[e];
                    }
                    sd += xor32(sd);
                    if ((tid & 63) == 0) blk_s[wv] = sd;
                    __syncthreads();
                    sd = blk_s[0];
                    for (int w = 1; w < 16; ++w) sd += blk_s[w];
                    __syncthreads();
#pragma unroll
                    for (int e = 0; e < ER; ++e)
                        if (validR(e)) dLd[e] -= fpm::fast_exp2(DUMMY - ud - pR[e]) * sd;
                }
            }
            // potentials in effect before step t (after step t - 2 on the same side, else 0);
            // unconditional loads at a clamped slot, then selects (per-thread conditional loads
            // here cost ~100 spilled VGPRs)
            {
                const bool have = t >= 2;
                const float* h = hist + (long)(have ? t - 2 : 0) * a.H;
                if (Rside) {
#pragma unroll
                    for (int e = 0; e < ER; ++e) {
                        const int r = tr + 32 * e;
                        const float v = h[min(r, a.H - 2)];
                        pR[e] = (have && r < boxPR) ? v : 0.f;
                    }
                } else {
#pragma unroll
                    for (int f = 0; f < EC; ++f) {
                        const int c = tc + 32 * f;
                        const float v = h[min(c, a.H - 2)];
                        pC[f] = (have && c < boxPC) ? v : 0.f;
                    }
                }
                if (algrow) ud = have ? h[a.H - 1] : 0.f;
            }
        }
        // dS = dL_0 / tau on the valid block, zeros in the padding (contiguous B x n1max x n2max)
        float* dsb = a.ds + (long)b * a.n1max * a.n2max;
        const float it_ = 1.f / a.tau;
        const int opr = a.contig_j ? a.n2max : 1, opc = a.contig_j ? 1 : a.n2max;
#pragma unroll
        for (int e = 0; e < ER; ++e) {
            const int pr = tr + 32 * e;
            if (pr >= boxPR) continue;
#pragma unroll
            for (int f = 0; f < EC; ++f) {
                const int pc = tc + 32 * f;
                if (pc >= boxPC) continue;
                dsb[pr * opr + pc * opc] = (pr < limPR && pc < limPC) ? DL(e, f) * it_ : 0.f;
            }
        }
}

// ---------------------------------------------------------------------------------------------
// Forward, max(n1max, n2max) <= 256: the log matrix itself is the register tile (L form).  Each
// step subtracts its lines' logsumexps from L, as the reference's ``L -= logsumexp(L, dim)``
// (pygmtools sinkhorn; oracle/ngm_oracle.py sinkhorn_m), instead of keeping S / tau and two
// potential vectors (sinkhorn_reg_kernel, kept for the backward's replay).  A step's subtraction is
// deferred into the next step's pass, which reads every entry anyway: one subtract, one v_exp and
// one add per entry and step, the subtract and the add on packed-f32 pairs (v_pk_add_f32), against
// two adds, a subtract, the v_exp and an add in the potential form.  The dummy rows (nd identical
// rows of value -100 over the valid algorithmic columns) are one log vector in LDS (``ldv``,
// indexed along the physical axis that carries the algorithmic columns).
typedef float f2 __attribute__((ext_vector_type(2)));


template <int ER, int EC, int NT>
__global__ __launch_bounds__(NT) void sinkhorn_lform_kernel(SinkArgs a) {
    static_assert(EC % 2 == 0, "column pairs");
    constexpr int NCOL = 32 * EC, EP = EC / 2, NP = ER > EC ? ER : EC;
    constexpr int TR = NT / 32, NW = NT / 64;   // thread rows, waves
    constexpr int NLD = (TR * ER > NCOL) ? TR * ER : NCOL;
    static_assert(NCOL <= NT, "one thread per column in the column reductions");
    __shared__ float red_m[NW][NCOL];
    __shared__ float red_s[NW][NCOL];
    __shared__ float fin[NCOL];
    __shared__ float ldv[NLD];
    __shared__ float ud_sh;
    __shared__ int redo_flag;

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int tr = tid >> 5, tc = tid & 31, wv = tid >> 6, lane = tid & 63;
    const int n1b = a.n1[b], n2b = a.n2[b];
    const bool transposed = n1b > n2b;
    const int R = transposed ? n2b : n1b;
    const int C = transposed ? n1b : n2b;
    const int nd = (a.dummy_row && C > R) ? (C - R) : 0;
    const float fnd = (float)nd;
    const int limPR = a.contig_j ? n1b : n2b;
    const int limPC = a.contig_j ? n2b : n1b;
    const int boxPR = a.contig_j ? a.n1max : a.n2max;
    const int boxPC = a.contig_j ? a.n2max : a.n1max;
    const bool u_on_R = (a.contig_j != 0) == (!transposed);
    const float DUMMY = -100.f * fpm::LOG2E_F;

    const float* in = a.in + (long)b * a.in_sb;
    const int ispr = (int)(a.contig_j ? a.in_si : a.in_sj);
    const int ispc = (int)(a.contig_j ? a.in_sj : a.in_si);

    // S / tau in log2 units as one multiply per entry (the IEEE division took ~10 VALU per entry)
    const float vscale = fpm::LOG2E_F / a.tau;
    // Column ownership: lane tc holds W = min(EC, 4) CONSECUTIVE columns per chunk, chunk c of
    // f = W c + w at pc = 32 W c + W tc + w, so a row's tile piece is one 16-B (W = 4) load / store
    // (64 scalar accesses + their address and bound arithmetic became 16 vector ones).  Column sums
    // are unchanged (same rows, same order); a row's sum visits its columns in another order.
    constexpr int W = EC >= 4 ? 4 : EC;
    static_assert(EC % W == 0 && (W == 4 || W == 2), "column chunks");
    f2 L[ER][EP];   // entry (tr + 32 e, pcol(tc, 2p + k)) in L[e][p][k]
    // loaded inside each side's path (run_steps below): nothing vector-valued is live across the
    // branch between the two compile-time step orders, so each is register-allocated on its own
    // (a tile loaded before the branch cost 33-47 VGPRs of scratch spills per thread)
    auto load_L = [&]() __attribute__((always_inline)) {
        const int tidL = opaque_i((int)threadIdx.x), trL = tidL >> 5, tcL = tidL & 31;
        // vector chunks: unit column stride, 16-B (8-B) aligned rows
        const bool vec = ispc == 1 && (ispr % W) == 0 && ((uintptr_t)in & (4 * W - 1)) == 0;
#pragma unroll
        for (int e = 0; e < ER; ++e) {
            const int pr = trL + TR * e;
#pragma unroll
            for (int c = 0; c < EC / W; ++c) {
                const int pc = 32 * W * c + W * tcL;
                float v[W];
                if (vec && pr < limPR && pc + W <= limPC) {
                    if constexpr (W == 4) {
                        const float4 q = *(const float4*)(in + pr * ispr + pc);
                        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
                    } else {
                        const float2 q = *(const float2*)(in + pr * ispr + pc);
                        v[0] = q.x; v[1] = q.y;
                    }
                } else {
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        v[w] = (pr < limPR && pc + w < limPC) ? in[pr * ispr + (pc + w) * ispc] : -INFINITY;
                }
                // the scale as packed multiplies (v_pk_mul_f32: the same fp32 products, -inf stays -inf)
#pragma unroll
                for (int w = 0; w < W; w += 2) L[e][(W * c + w) / 2] = f2{v[w], v[w + 1]} * f2{vscale, vscale};
            }
        }
    };
    // pending deltas of the last step (row deltas pd[e] after a row-side step, column deltas pd[f]
    // after a column-side step), subtracted by the next pass
    float pd[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) pd[k] = 0.f;
    // dummy log vector along the algorithmic-column axis: pr (u_on_R false) or pc (u_on_R true)
    const int limY = u_on_R ? limPC : limPR;
    for (int k = tid; k < NLD; k += NT) ldv[k] = (nd > 0 && k < limY) ? DUMMY : -INFINITY;
    if (tid == 0) redo_flag = 0;
    __syncthreads();

    auto ok_s = [](float x) { return x >= 0x1p-30f && x <= 0x1p30f; };
    // The bounds tests are recomputed where they are used, from copies the compiler cannot see
    // through: hoisted and shared between the loads, the steps and the stores, the 128 per-entry
    // masks stayed live for the whole kernel (SGPR spills into VGPR lanes, then VGPR spills).
    auto opaque = [](int v) { asm volatile("" : "+v"(v)); return v; };
#define pc_of(f) (32 * W * ((f) / W) + W * tc + ((f) % W))   // f = 2p + k
    // Thread coordinates, re-derived inside each step for the same reason: loop-invariant lane
    // indices, row numbers and LDS addresses hoisted out of the step loop held ~30 VGPRs.
#define SK_LOCAL_COORDS                                                       \
    const int tid = opaque((int)threadIdx.x);                                 \
    const int tr = tid >> 5, tc = tid & 31, wv = tid >> 6, lane = tid & 63;   \
    (void)tr; (void)tc; (void)wv; (void)lane;

    // Row side: every physical row pr minus its lse over pc (+ the dummy term when the pr axis
    // carries the algorithmic columns, add_dummy).  Pending column deltas come in.
    auto step_R = [&](bool add_dummy, bool fast) __attribute__((always_inline)) {
        SK_LOCAL_COORDS
        const int limR = opaque(limPR);
        // the pending column deltas first, in one unconditional pass (L is written in one place
        // per step: updates inside the fast / fallback branches merged into register copies)
        {
            f2 dc[EP];
#pragma unroll
            for (int p = 0; p < EP; ++p) dc[p] = f2{pd[2 * p], pd[2 * p + 1]};
#pragma unroll
            for (int e = 0; e < ER; ++e)
#pragma unroll
                for (int p = 0; p < EP; ++p) L[e][p] -= dc[p];
        }
        if (fast) {
            float s[ER];
#pragma unroll
            for (int e = 0; e < ER; ++e) {
                f2 acc = {fpm::fast_exp2(L[e][0].x), fpm::fast_exp2(L[e][0].y)};
#pragma unroll
                for (int p = 1; p < EP; ++p) acc += f2{fpm::fast_exp2(L[e][p].x), fpm::fast_exp2(L[e][p].y)};
                s[e] = acc.x + acc.y;
            }
#pragma unroll
            for (int e = 0; e < ER; ++e) s[e] = lane32_sum(s[e]);
            bool bad = false;
#pragma unroll
            for (int e = 0; e < ER; ++e) {
                const int pr = tr + TR * e;
                if (add_dummy) s[e] += fnd * fpm::fast_exp2(ldv[pr < NLD ? pr : 0]);
                bad |= pr < limR && !ok_s(s[e]);
            }
            if (__ballot(bad) == 0ull) {
#pragma unroll
                for (int e = 0; e < ER; ++e) {
                    const int pr = tr + TR * e;
                    pd[e] = pr < limR ? fpm::fast_log2(s[e]) : 0.f;
                    if (add_dummy && tc == 0 && pr < limR) ldv[pr] -= pd[e];
                }
                return;
            }
        }
        // max-shifted lse on L (pending deltas already applied)
#pragma unroll
        for (int e = 0; e < ER; ++e) {
            const int pr = tr + TR * e;
            float m = -INFINITY;
#pragma unroll
            for (int p = 0; p < EP; ++p) m = fmaxf(m, fmaxf(L[e][p].x, L[e][p].y));
            m = lane32_max(m);
            const float ld = add_dummy ? ldv[pr < NLD ? pr : 0] : -INFINITY;
            m = fmaxf(m, ld);
            float t = 0.f;
            if (m != -INFINITY) {
#pragma unroll
                for (int p = 0; p < EP; ++p)
                    t += fpm::fast_exp2(L[e][p].x - m) + fpm::fast_exp2(L[e][p].y - m);
            }
            t = lane32_sum(t);
            if (add_dummy && m != -INFINITY) t += fnd * fpm::fast_exp2(ld - m);
            pd[e] = (m == -INFINITY || pr >= limR) ? 0.f : m + fpm::fast_log2(t);
            if (add_dummy && tc == 0 && pr < limR) ldv[pr] -= pd[e];
        }
    };

    // Column side: every physical column pc minus its lse over pr (+ the dummy term when the pc
    // axis carries the algorithmic columns).  Pending row deltas come in; the 32 thread rows of a
    // column reduce through one lane swap and LDS.
    auto step_C = [&](bool add_dummy, bool fast) __attribute__((always_inline)) {
        SK_LOCAL_COORDS
        const int limC = opaque(limPC);
#pragma unroll
        for (int e = 0; e < ER; ++e) {
            const f2 dr = {pd[e], pd[e]};
#pragma unroll
            for (int p = 0; p < EP; ++p) L[e][p] -= dr;
        }
        if (fast) {
            f2 cs[EP];
#pragma unroll
            for (int p = 0; p < EP; ++p) cs[p] = f2{fpm::fast_exp2(L[0][p].x), fpm::fast_exp2(L[0][p].y)};
#pragma unroll
            for (int e = 1; e < ER; ++e)
#pragma unroll
                for (int p = 0; p < EP; ++p) cs[p] += f2{fpm::fast_exp2(L[e][p].x), fpm::fast_exp2(L[e][p].y)};
#pragma unroll
            for (int p = 0; p < EP; ++p) {
                const float s0 = cs[p].x + xor32(cs[p].x), s1 = cs[p].y + xor32(cs[p].y);
                if (lane < 32) {
                    red_s[wv][pc_of(2 * p)] = s0;
                    red_s[wv][pc_of(2 * p + 1)] = s1;
                }
            }
            __syncthreads();
            if (tid < NCOL) {
                float s = red_s[0][tid];
                for (int w = 1; w < NW; ++w) s += red_s[w][tid];
                if (add_dummy) s += fnd * fpm::fast_exp2(ldv[tid < NLD ? tid : 0]);
                if (tid >= limC) fin[tid] = 0.f;
                else if (ok_s(s)) fin[tid] = fpm::fast_log2(s);
                else redo_flag = 1;
            }
            __syncthreads();
            const bool redo = redo_flag != 0;
            if (!redo) {
#pragma unroll
                for (int f = 0; f < EC; ++f) pd[f] = fin[pc_of(f)];
                if (add_dummy && tid < NCOL && tid < limC) ldv[tid] -= fin[tid];
                return;   // the next read of ldv / redo_flag is behind a barrier
            }
        }
        // max-shifted: per-thread (max, sum) over its ER rows, combined over the column
#pragma unroll
        for (int f = 0; f < EC; ++f) {
            const int p = f >> 1;
            float m = -INFINITY;
#pragma unroll
            for (int e = 0; e < ER; ++e) m = fmaxf(m, (f & 1) ? L[e][p].y : L[e][p].x);
            float s = 0.f;
            if (m != -INFINITY) {
#pragma unroll
                for (int e = 0; e < ER; ++e) s += fpm::fast_exp2(((f & 1) ? L[e][p].y : L[e][p].x) - m);
            }
            float mo = xor32(m), so = xor32(s);
            lse_combine(m, s, mo, so);
            if (lane < 32) {
                red_m[wv][pc_of(f)] = m;
                red_s[wv][pc_of(f)] = s;
            }
        }
        __syncthreads();
        if (tid < NCOL) {
            float m = red_m[0][tid], s = red_s[0][tid];
            for (int w = 1; w < NW; ++w) lse_combine(m, s, red_m[w][tid], red_s[w][tid]);
            if (add_dummy) lse_combine(m, s, ldv[tid < NLD ? tid : 0], fnd);
            const float d = (m == -INFINITY || tid >= limC) ? 0.f : m + fpm::fast_log2(s);
            fin[tid] = d;
            if (add_dummy && tid < limC) ldv[tid] -= d;
        }
        __syncthreads();
#pragma unroll
        for (int f = 0; f < EC; ++f) pd[f] = fin[pc_of(f)];
        if (tid == 0) redo_flag = 0;    // every thread read it before the barrier above
    };

    // dummy rows: ldv minus its lse over the valid algorithmic columns (one wave; rare path)
    auto update_dummy = [&]() __attribute__((always_inline)) {
        SK_LOCAL_COORDS
        __syncthreads();
        if (wv == 0) {
            float m = -INFINITY;
            for (int k = lane; k < limY; k += 64) m = fmaxf(m, ldv[k]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
            float s = 0.f;
            for (int k = lane; k < limY; k += 64) s += fpm::fast_exp2(ldv[k] - m);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
            const float d = m == -INFINITY ? 0.f : m + fpm::fast_log2(s);
            for (int k = lane; k < limY; k += 64) ldv[k] -= d;
        }
        __syncthreads();
    };
    (void)ud_sh;

    // The output: exp2(L - the last step's pending deltas), with the side of the last step a
    // compile-time constant and the coordinates re-derived here (values kept live across the step
    // loop -- thread coordinates, a runtime choice between the row and column deltas -- were spilled
    // to scratch: 49 VGPRs per thread stored and reloaded per launch)
    auto store_out = [&](auto lastr) __attribute__((always_inline)) {
        constexpr bool LR = decltype(lastr)::value;
        float* out = a.out + (long)b * a.out_sb;
        const int opr = (int)(a.contig_j ? a.out_si : a.out_sj);
        const int opc = (int)(a.contig_j ? a.out_sj : a.out_si);
        const int oPR = opaque(limPR), oPC = opaque(limPC), obPR = opaque(boxPR), obPC = opaque(boxPC);
        const int tidE = opaque((int)threadIdx.x), trE = tidE >> 5, tcE = tidE & 31;
        const bool vec = opc == 1 && (opr % W) == 0 && ((uintptr_t)out & (4 * W - 1)) == 0;
#pragma unroll
        for (int e = 0; e < ER; ++e) {
            const int pr = trE + TR * e;
            if (pr >= obPR) continue;
#pragma unroll
            for (int c = 0; c < EC / W; ++c) {
                const int pc = 32 * W * c + W * tcE;
                float v[W];
                const bool full = pr < oPR && pc + W <= oPC;     // the whole chunk valid: no per-entry test
#pragma unroll
                for (int w = 0; w < W; w += 2) {
                    // the pending deltas as packed subtracts (v_pk_add_f32), then the exps
                    const int f = W * c + w;
                    const f2 t = L[e][f >> 1] - (LR ? f2{pd[e], pd[e]} : f2{pd[f], pd[f + 1]});
                    v[w] = fpm::fast_exp2(t.x);
                    v[w + 1] = fpm::fast_exp2(t.y);
                }
                if (!full) {
#pragma unroll
                    for (int w = 0; w < W; ++w) v[w] = (pr < oPR && pc + w < oPC) ? v[w] : 0.f;
                }
                if (vec && pc + W <= obPC) {
                    if constexpr (W == 4) *(float4*)(out + pr * opr + pc) = make_float4(v[0], v[1], v[2], v[3]);
                    else *(float2*)(out + pr * opr + pc) = make_float2(v[0], v[1]);
                } else {
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        if (pc + w < obPC) out[pr * opr + (pc + w) * opc] = v[w];
                }
            }
        }
    };

    // Steps in (row, column) pairs with the physical sides fixed at compile time: L then flows
    // through straight-line code (a runtime choice of side per step merged the two updated tiles
    // at every join -- register copies and spills).  Row steps (even) normalise the algorithmic
    // rows; column steps (odd) count the dummy rows.  Ends with the store for the last step's side.
    auto run_steps = [&](auto rfirst) __attribute__((always_inline)) {
        constexpr bool RF = decltype(rfirst)::value;
        load_L();
        int it = 0;
        for (; it + 1 < a.iters; it += 2) {
            const bool fast0 = it > 0 && a.fast;
            if constexpr (RF) step_R(false, fast0); else step_C(false, fast0);
            if (nd > 0) update_dummy();
            if constexpr (RF) step_C(nd > 0, a.fast != 0); else step_R(nd > 0, a.fast != 0);
        }
        if (it < a.iters) {
            const bool fast0 = it > 0 && a.fast;
            if constexpr (RF) step_R(false, fast0); else step_C(false, fast0);
            if (nd > 0) update_dummy();
            store_out(std::integral_constant<bool, RF>{});
            return;
        }
        store_out(std::integral_constant<bool, !RF>{});
    };
#undef pc_of
#undef SK_LOCAL_COORDS
    if (u_on_R) run_steps(std::true_type{});
    else run_steps(std::false_type{});
}

// ---------------------------------------------------------------------------------------------
// Large blocks (max(n1max, n2max) > 256, e.g. n = 512): the block no longer fits the register file,
// so every half-iteration streams the pair's block from L2 / HBM (1 MB at n = 512) while the
// potentials stay in LDS.  Same algorithm and semantics as sinkhorn_reg_kernel; the per-thread
// logsumexps are single-pass (online max rescaling).
// Physical axes: "a" = the strided axis, "c" = the unit-stride axis of the input.
constexpr int SK_MAXN = 2048;

__device__ __forceinline__ void lse_push(float& m, float& s, float x) {
    if (x > m) {
        s = s * fpm::fast_exp2(m - x) + 1.f;
        m = x;
    } else {
        s += fpm::fast_exp2(x - m);
    }
}

typedef unsigned int sk_u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(1024) void sinkhorn_stream_kernel(SinkArgs a) {
    __shared__ __attribute__((aligned(16))) float potA[SK_MAXN], potC[SK_MAXN];
    __shared__ float4 red4[1024];
    __shared__ float red_m[1024], red_s[1024];
    __shared__ float ud_sh;
    __shared__ __attribute__((aligned(16))) float newC[SK_MAXN], xmax[SK_MAXN];
    __shared__ int redo_sh, xfail_sh;
    // split launches: XCD x = block % 8 takes pairs x, x + 8, ...; a pair's G sibling workgroups are
    // consecutive in that XCD's dispatch order (its exchanges stay in one L2, and a waiting sibling
    // only ever waits for workgroups dispatched before or right after it)
    const int G = a.split > 1 ? a.split : 1;
    int b = blockIdx.x, j = 0;
    if (G > 1) {
        const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
        b = (k / G) * 8 + x;
        j = k % G;
        if (b >= a.B) return;
    }
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n1b = a.n1[b], n2b = a.n2[b];
    const bool transposed = n1b > n2b;
    const int R = transposed ? n2b : n1b, C = transposed ? n1b : n2b;
    const int nd = (a.dummy_row && C > R) ? (C - R) : 0;
    const float DUMMY = -100.f * fpm::LOG2E_F;
    const float scale = fpm::LOG2E_F / a.tau;
    const int limA = a.contig_j ? n1b : n2b, limC = a.contig_j ? n2b : n1b;
    const int boxA = a.contig_j ? a.n1max : a.n2max, boxC = a.contig_j ? a.n2max : a.n1max;
    const bool u_on_A = (a.contig_j != 0) == (!transposed);
    const float* in = a.in + (long)b * a.in_sb;
    const long sA = a.contig_j ? a.in_si : a.in_sj, sC = a.contig_j ? a.in_sj : a.in_si;
    const float vscale = fpm::LOG2E_F / a.tau;   // one multiply per element read (not a division)
    auto val = [&](int ia, int ic) { return in[ia * sA + ic * sC] * vscale; };
    // 16-B loads along c for the fast steps: unit-stride c, 16-B aligned rows, whole quads
    // (a.fast == 2 keeps the scalar loads: A/B switch)
    const bool vec = sC == 1 && (sA & 3) == 0 && ((unsigned long)in & 15) == 0 && (limC & 3) == 0 &&
                     a.fast == 1;
    auto e4 = [&](float4 v, float4 p, float sh) {       // sum of exp2(v * vscale - p - sh) over 4
        return fpm::fast_exp2(v.x * vscale - p.x - sh) + fpm::fast_exp2(v.y * vscale - p.y - sh) +
               fpm::fast_exp2(v.z * vscale - p.z - sh) + fpm::fast_exp2(v.w * vscale - p.w - sh);
    };
    (void)scale;
    // Split pairs (G > 1; square or dummy-free pairs on the 16-B path, >= 64 lines per workgroup):
    // sibling j owns the a-lines [a_lo, a_hi) -- their row potentials, their share of every column
    // sum, their output rows -- and keeps the whole column-potential vector.  A column step
    // exchanges the G partial column sums (or (max, sum) pairs) through global memory; every
    // sibling combines them in sibling order, so all hold the same potentials and take the same
    // fallback decisions.  Other pairs run whole on sibling 0 (the rest return).
    // (a pair with fewer than 64 G lines uses floor(lines / 64) siblings: its own size decides)
    const int gcap = limA / 64 < G ? limA / 64 : G;
    const bool split = G > 1 && vec && a.rw > 1 && nd == 0 && gcap >= 2;
    if (G > 1 && (!split || j >= gcap) && j != 0) return;
    const int GP = split ? gcap : 1, jj = split ? j : 0;
    const int a_lo = (int)((long)limA * jj / GP), a_hi = (int)((long)limA * (jj + 1) / GP);
    int xr = 0;   // exchange rounds so far (the same count in every sibling)
    for (int k = tid; k < SK_MAXN; k += 1024) { potA[k] = 0.f; potC[k] = 0.f; }
    if (tid == 0) { ud_sh = 0.f; redo_sh = 0; xfail_sh = 0; }
    __syncthreads();

    // One exchange round (cdna_hip_programming.md Guideline 16, R1 / table row 1): the partial sums
    // newC[0, limC) (and the partial maxima xmax when `two`) leave as 16-B sc1 stores into this
    // sibling's slot, every wave drains its stores, a barrier, then ONE lane adds to the pair's
    // arrival counter (agent scope) and polls it (relaxed sc1 loads, bounded: a missing sibling sets
    // xfail and the outputs become NaN instead of the launch hanging), a barrier; the slots are then
    // read with sc1 buffer loads only (ld_slot; FPM_SK_XACQ=1 adds an agent acquire fence).  Slots
    // alternate between two buffers: a sibling's round r + 2 store can only follow every sibling's
    // round r + 1 arrival, which follows its reads of round r.
    auto slot_of = [&](int g, int r) { return a.xbuf + (((long)b * G + g) * 2 + (r & 1)) * a.xslot; };
    // a slot's 16 B at float offset `off`: an sc1 buffer load (bypasses this CU's L1; the Guideline-16
    // table's row 1 -- sc1 stores, one lane's agent-scope counter add after every storing wave's drain
    // and a barrier, one lane's sc1 poll, every load of the bytes sc1, one workgroup per CU -- needs no
    // acquire fence then; a.xacq = 1 keeps the fence anyway)
    auto ld_slot = [&](int g, int r, long off) {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)slot_of(g, r), (short)0, (int)(a.xslot * 4), 0x00020000);
        const sk_u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off * 4), 0, 16);
        return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
    };
    auto exchange = [&](bool two) {
        float* slot = slot_of(j, xr);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)slot, (short)0, (int)(a.xslot * 4), 0x00020000);
        const int nq = limC >> 2;
        for (int q = tid; q < nq; q += 1024) {
            const float4 v = *(const float4*)&newC[4 * q];
            __builtin_amdgcn_raw_buffer_store_b128(
                (sk_u32x4){__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)},
                rs, 16 * q, 0, 16);
            if (two) {
                const float4 m = *(const float4*)&xmax[4 * q];
                __builtin_amdgcn_raw_buffer_store_b128(
                    (sk_u32x4){__float_as_uint(m.x), __float_as_uint(m.y), __float_as_uint(m.z), __float_as_uint(m.w)},
                    rs, (int)(a.xslot / 2) * 4 + 16 * q, 0, 16);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_fetch_add(a.xcnt + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int target = GP * (xr + 1);
            unsigned spins = 0;
            // bounded: ~2^20 polls (about a second); after one failure later rounds do not wait
            while (!xfail_sh && __hip_atomic_load(a.xcnt + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 20)) xfail_sh = 1;
            }
            if (a.xacq) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the loads below
            }
        }
        __syncthreads();
        ++xr;
    };

    // Shifted single-pass lse (fast, every step after the first; as in sinkhorn_reg_kernel): after
    // a normalisation along one axis every entry is <= 0, so the other axis' lse is shifted by the
    // line's previous potential -- one exp and one add per element, a plain sum reduction.  A sum
    // outside [2^-30, 2^30] falls back to the online max-rescaled form (per row on the c side; the
    // whole step on the a side, like the register kernel).
    auto ok_s = [](float x) { return x >= 0x1p-30f && x <= 0x1p30f; };
    // potA[ia] = lse_c(val - potC[c]) (+ nd * exp(DUMMY - ud)): one wave per ia, lanes along c
    auto along_c = [&](bool add_dummy, bool fast) {
        const float ud = ud_sh;
        auto multi_rows = [&](auto rwc, bool shifted) {
            // SK_RW rows per wave at once (rows wv + 16 t): their 16-B loads in flight together, the
            // row sums reduced on DPP / v_permlane (fpm::wave_sum_dpp) instead of six ds_bpermute
            // round trips each; a row whose shifted sum leaves [2^-30, 2^30] takes the online form
            // below.  (The single-row loop was load- and shuffle-latency bound: ~16 GB/s per CU.)
            constexpr int RW = decltype(rwc)::value;
            const int span = a_hi - a_lo;                   // this workgroup's a-lines
            const int nrow = span > wv ? (span - wv + 15) / 16 : 0;
            for (int t0 = 0; t0 < nrow; t0 += RW) {
                float sh[RW], sm[RW];
                const float* rp[RW];
#pragma unroll
                for (int r = 0; r < RW; ++r) {
                    const int ia = a_lo + wv + 16 * (t0 + r < nrow ? t0 + r : t0);
                    sh[r] = potA[ia];
                    sm[r] = 0.f;
                    rp[r] = in + (long)ia * sA;
                }
                if (!shifted) {
                    // first step (no previous potential to shift by): the row max of val - potC in
                    // a pass of its own, then the max-shifted sum -- two vector passes instead of
                    // the online rescale on scalar loads
#pragma unroll
                    for (int r = 0; r < RW; ++r) sh[r] = -INFINITY;
                    for (int ic = 4 * lane; ic < limC; ic += 256) {
                        const float4 pc = *(const float4*)&potC[ic];
#pragma unroll
                        for (int r = 0; r < RW; ++r) {
                            const float4 v = *(const float4*)(rp[r] + ic);
                            sh[r] = fmaxf(fmaxf(fmaxf(sh[r], v.x * vscale - pc.x), fmaxf(v.y * vscale - pc.y,
                                          v.z * vscale - pc.z)), v.w * vscale - pc.w);
                        }
                    }
#pragma unroll
                    for (int r = 0; r < RW; ++r) sh[r] = fpm::warp_max(sh[r]);
                }
                for (int ic = 4 * lane; ic < limC; ic += 256) {
                    const float4 pc = *(const float4*)&potC[ic];
                    float4 v[RW];
#pragma unroll
                    for (int r = 0; r < RW; ++r) v[r] = *(const float4*)(rp[r] + ic);
#pragma unroll
                    for (int r = 0; r < RW; ++r) sm[r] += e4(v[r], pc, sh[r] == -INFINITY ? 0.f : sh[r]);
                }
#pragma unroll
                for (int r = 0; r < RW; ++r) {
                    if (t0 + r >= nrow) break;
                    const int ia = a_lo + wv + 16 * (t0 + r);
                    if (!shifted) {
                        float m = sh[r], s2 = fpm::wave_sum_dpp(sm[r]);
                        if (m == -INFINITY) s2 = 0.f;
                        if (add_dummy) lse_combine(m, s2, DUMMY - ud, (float)nd);
                        if (lane == 0) potA[ia] = (m == -INFINITY) ? 0.f : m + fpm::fast_log2(s2);
                        continue;
                    }
                    float sr = fpm::wave_sum_dpp(sm[r]);
                    if (add_dummy) sr += (float)nd * fpm::fast_exp2(DUMMY - ud - sh[r]);
                    if (ok_s(sr)) {
                        if (lane == 0) potA[ia] = sh[r] + fpm::fast_log2(sr);
                        continue;
                    }
                    // out of range (wave-uniform): this row's exact max, then the max-shifted sum,
                    // both on 16-B loads
                    float m = -INFINITY, s2 = 0.f;
                    for (int ic = 4 * lane; ic < limC; ic += 256) {
                        const float4 pc = *(const float4*)&potC[ic];
                        const float4 v = *(const float4*)(rp[r] + ic);
                        m = fmaxf(fmaxf(fmaxf(m, v.x * vscale - pc.x), fmaxf(v.y * vscale - pc.y, v.z * vscale - pc.z)),
                                  v.w * vscale - pc.w);
                    }
                    m = fpm::warp_max(m);
                    for (int ic = 4 * lane; ic < limC; ic += 256)
                        s2 += e4(*(const float4*)(rp[r] + ic), *(const float4*)&potC[ic], m == -INFINITY ? 0.f : m);
                    s2 = m == -INFINITY ? 0.f : fpm::wave_sum_dpp(s2);
                    if (add_dummy) lse_combine(m, s2, DUMMY - ud, (float)nd);
                    if (lane == 0) potA[ia] = (m == -INFINITY) ? 0.f : m + fpm::fast_log2(s2);
                }
            }
        };
        if (vec && a.rw > 1 && (fast || a.fast)) {
            if (a.rw >= 4) multi_rows(std::integral_constant<int, 4>{}, fast);
            else multi_rows(std::integral_constant<int, 2>{}, fast);
            __syncthreads();
            return;
        }
        for (int ia = wv; ia < limA; ia += 16) {
            if (fast && vec) {
                const float sh = potA[ia];
                const float* row = in + (long)ia * sA;
                float s0 = 0.f, s1 = 0.f;
                int ic = 4 * lane;
#pragma unroll 2
                for (; ic + 256 < limC; ic += 512) {
                    s0 += e4(*(const float4*)(row + ic), *(const float4*)&potC[ic], sh);
                    s1 += e4(*(const float4*)(row + ic + 256), *(const float4*)&potC[ic + 256], sh);
                }
                if (ic < limC) s0 += e4(*(const float4*)(row + ic), *(const float4*)&potC[ic], sh);
                float s = s0 + s1;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                if (add_dummy) s += (float)nd * fpm::fast_exp2(DUMMY - ud - sh);
                if (ok_s(s)) {
                    if (lane == 0) potA[ia] = sh + fpm::fast_log2(s);
                    continue;
                }
            } else if (fast) {
                const float sh = potA[ia];
                float s0 = 0.f, s1 = 0.f;
                int ic = lane;
#pragma unroll 4
                for (; ic + 64 < limC; ic += 128) {
                    s0 += fpm::fast_exp2(val(ia, ic) - potC[ic] - sh);
                    s1 += fpm::fast_exp2(val(ia, ic + 64) - potC[ic + 64] - sh);
                }
                if (ic < limC) s0 += fpm::fast_exp2(val(ia, ic) - potC[ic] - sh);
                float s = s0 + s1;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                if (add_dummy) s += (float)nd * fpm::fast_exp2(DUMMY - ud - sh);
                if (ok_s(s)) {                        // wave-uniform (s is reduced over the wave)
                    if (lane == 0) potA[ia] = sh + fpm::fast_log2(s);
                    continue;
                }
            }
            float m = -INFINITY, s = 0.f;
#pragma unroll 8
            for (int ic = lane; ic < limC; ic += 64) lse_push(m, s, val(ia, ic) - potC[ic]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                float mo = __shfl_xor(m, o), so = __shfl_xor(s, o);
                lse_combine(m, s, mo, so);
            }
            if (add_dummy) lse_combine(m, s, DUMMY - ud, (float)nd);
            if (lane == 0) potA[ia] = (m == -INFINITY) ? 0.f : m + fpm::fast_log2(s);
        }
        __syncthreads();
    };
    // potC[ic] = lse_a(val - potA[a]) (+ dummy): thread groups along a, threads along c (coalesced)
    auto along_a = [&](bool add_dummy, bool fast) {
        const float ud = ud_sh;
        const int cpad = (limC + 63) / 64 * 64;
        const int groups = cpad >= 1024 ? 1 : 1024 / cpad;
        if (split) {
            // this sibling's share of every column sum over its a-lines, exchanged and combined in
            // sibling order (no dummy rows here: nd == 0)
            const int nq = limC >> 2, qpad = (nq + 63) / 64 * 64;
            const int groups4 = qpad >= 1024 ? 1 : 1024 / qpad;
            if (fast) {
                for (int q0 = 0; q0 < nq; q0 += 1024) {
                    const int q = q0 + (groups4 == 1 ? tid : tid % qpad), grp = groups4 == 1 ? 0 : tid / qpad;
                    const int ic = 4 * q;
                    float4 sh = make_float4(0.f, 0.f, 0.f, 0.f), acc = sh;
                    if (q < nq) sh = *(const float4*)&potC[ic];
                    if (q < nq && grp < groups4) {
#pragma unroll 8
                        for (int ia = a_lo + grp; ia < a_hi; ia += groups4) {
                            const float4 v = *(const float4*)(in + (long)ia * sA + ic);
                            const float pa = potA[ia];
                            acc.x += fpm::fast_exp2(v.x * vscale - pa - sh.x);
                            acc.y += fpm::fast_exp2(v.y * vscale - pa - sh.y);
                            acc.z += fpm::fast_exp2(v.z * vscale - pa - sh.z);
                            acc.w += fpm::fast_exp2(v.w * vscale - pa - sh.w);
                        }
                    }
                    red4[tid] = acc;
                    __syncthreads();
                    if (grp == 0 && q < nq) {
                        for (int g = 1; g < groups4; ++g) {
                            const float4 o = red4[tid + g * qpad];
                            acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
                        }
                        *(float4*)&newC[ic] = acc;
                    }
                    __syncthreads();
                }
                exchange(false);
                for (int q = tid; q < nq; q += 1024) {
                    float4 t = ld_slot(0, xr - 1, 4 * q);
                    for (int g = 1; g < GP; ++g) {
                        const float4 o = ld_slot(g, xr - 1, 4 * q);
                        t.x += o.x; t.y += o.y; t.z += o.z; t.w += o.w;
                    }
                    const float4 sh = *(const float4*)&potC[4 * q];
                    const float sv[4] = {t.x, t.y, t.z, t.w}, hv[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (ok_s(sv[k])) newC[4 * q + k] = hv[k] + fpm::fast_log2(sv[k]);
                        else redo_sh = 1;
                    }
                }
                __syncthreads();
                const bool redo = redo_sh != 0;          // the same in every sibling (same totals)
                __syncthreads();
                if (!redo) {
                    for (int k = tid; k < limC; k += 1024) potC[k] = newC[k];
                    __syncthreads();
                    return;
                }
                if (tid == 0) redo_sh = 0;
            }
            // exact form: each sibling's column max over its lines, the sum shifted by it; combined
            // as (max, sum) pairs in sibling order
            for (int q0 = 0; q0 < nq; q0 += 1024) {
                const int q = q0 + (groups4 == 1 ? tid : tid % qpad), grp = groups4 == 1 ? 0 : tid / qpad;
                const int ic = 4 * q;
                const bool act = q < nq && grp < groups4;
                float4 mx = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
                if (act)
#pragma unroll 8
                    for (int ia = a_lo + grp; ia < a_hi; ia += groups4) {
                        const float4 v = *(const float4*)(in + (long)ia * sA + ic);
                        const float pa = potA[ia];
                        mx.x = fmaxf(mx.x, v.x * vscale - pa);
                        mx.y = fmaxf(mx.y, v.y * vscale - pa);
                        mx.z = fmaxf(mx.z, v.z * vscale - pa);
                        mx.w = fmaxf(mx.w, v.w * vscale - pa);
                    }
                red4[tid] = mx;
                __syncthreads();
                if (q < nq) {
                    const int t0 = groups4 == 1 ? tid : tid % qpad;
                    for (int g = 0; g < groups4; ++g) {
                        const float4 o = red4[t0 + g * qpad];
                        mx.x = fmaxf(mx.x, o.x); mx.y = fmaxf(mx.y, o.y); mx.z = fmaxf(mx.z, o.z); mx.w = fmaxf(mx.w, o.w);
                    }
                }
                __syncthreads();
                const float4 sh = make_float4(mx.x == -INFINITY ? 0.f : mx.x, mx.y == -INFINITY ? 0.f : mx.y,
                                              mx.z == -INFINITY ? 0.f : mx.z, mx.w == -INFINITY ? 0.f : mx.w);
                float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                if (act)
#pragma unroll 8
                    for (int ia = a_lo + grp; ia < a_hi; ia += groups4) {
                        const float4 v = *(const float4*)(in + (long)ia * sA + ic);
                        const float pa = potA[ia];
                        acc.x += fpm::fast_exp2(v.x * vscale - pa - sh.x);
                        acc.y += fpm::fast_exp2(v.y * vscale - pa - sh.y);
                        acc.z += fpm::fast_exp2(v.z * vscale - pa - sh.z);
                        acc.w += fpm::fast_exp2(v.w * vscale - pa - sh.w);
                    }
                red4[tid] = acc;
                __syncthreads();
                if (grp == 0 && q < nq) {
                    for (int g = 1; g < groups4; ++g) {
                        const float4 o = red4[tid + g * qpad];
                        acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
                    }
                    *(float4*)&newC[ic] = acc;
                    *(float4*)&xmax[ic] = mx;
                }
                __syncthreads();
            }
            exchange(true);
            for (int q = tid; q < nq; q += 1024) {
                float4 t = ld_slot(0, xr - 1, 4 * q), m4 = ld_slot(0, xr - 1, a.xslot / 2 + 4 * q);
                float sv[4] = {t.x, t.y, t.z, t.w}, mv[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (mv[k] == -INFINITY) sv[k] = 0.f;
                for (int g = 1; g < GP; ++g) {
                    const float4 to = ld_slot(g, xr - 1, 4 * q), mo = ld_slot(g, xr - 1, a.xslot / 2 + 4 * q);
                    const float so[4] = {to.x, to.y, to.z, to.w}, mov[4] = {mo.x, mo.y, mo.z, mo.w};
#pragma unroll
                    for (int k = 0; k < 4; ++k) lse_combine(mv[k], sv[k], mov[k], mov[k] == -INFINITY ? 0.f : so[k]);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) newC[4 * q + k] = (mv[k] == -INFINITY) ? 0.f : mv[k] + fpm::fast_log2(sv[k]);
            }
            __syncthreads();
            for (int k = tid; k < limC; k += 1024) potC[k] = newC[k];
            __syncthreads();
            return;
        }
        if (!fast && vec && a.rw > 1 && a.fast) {
            // first step: per column quad the max over the rows of val - potA, then the max-shifted
            // sum (two vector passes; row groups combined through LDS), as in along_c's first step
            const int nq = limC >> 2, qpad = (nq + 63) / 64 * 64;
            const int groups4 = qpad >= 1024 ? 1 : 1024 / qpad;
            for (int q0 = 0; q0 < nq; q0 += 1024) {
                const int q = q0 + (groups4 == 1 ? tid : tid % qpad), grp = groups4 == 1 ? 0 : tid / qpad;
                const int ic = 4 * q;
                const bool act = q < nq && grp < groups4;
                float4 mx = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
                if (act)
#pragma unroll 8
                    for (int ia = grp; ia < limA; ia += groups4) {
                        const float4 v = *(const float4*)(in + (long)ia * sA + ic);
                        const float pa = potA[ia];
                        mx.x = fmaxf(mx.x, v.x * vscale - pa);
                        mx.y = fmaxf(mx.y, v.y * vscale - pa);
                        mx.z = fmaxf(mx.z, v.z * vscale - pa);
                        mx.w = fmaxf(mx.w, v.w * vscale - pa);
                    }
                red4[tid] = mx;
                __syncthreads();
                if (q < nq) {
                    const int t0 = groups4 == 1 ? tid : tid % qpad;
                    for (int g = 0; g < groups4; ++g) {
                        const float4 o = red4[t0 + g * qpad];
                        mx.x = fmaxf(mx.x, o.x); mx.y = fmaxf(mx.y, o.y); mx.z = fmaxf(mx.z, o.z); mx.w = fmaxf(mx.w, o.w);
                    }
                }
                __syncthreads();
                const float4 sh = make_float4(mx.x == -INFINITY ? 0.f : mx.x, mx.y == -INFINITY ? 0.f : mx.y,
                                              mx.z == -INFINITY ? 0.f : mx.z, mx.w == -INFINITY ? 0.f : mx.w);
                float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                if (act)
#pragma unroll 8
                    for (int ia = grp; ia < limA; ia += groups4) {
                        const float4 v = *(const float4*)(in + (long)ia * sA + ic);
                        const float pa = potA[ia];
                        acc.x += fpm::fast_exp2(v.x * vscale - pa - sh.x);
                        acc.y += fpm::fast_exp2(v.y * vscale - pa - sh.y);
                        acc.z += fpm::fast_exp2(v.z * vscale - pa - sh.z);
                        acc.w += fpm::fast_exp2(v.w * vscale - pa - sh.w);
                    }
                red4[tid] = acc;
                __syncthreads();
                if (grp == 0 && q < nq) {
                    for (int g = 1; g < groups4; ++g) {
                        const float4 o = red4[tid + g * qpad];
                        acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
                    }
                    const float mv[4] = {mx.x, mx.y, mx.z, mx.w}, sv[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        float m = mv[k], sk = m == -INFINITY ? 0.f : sv[k];
                        if (add_dummy) lse_combine(m, sk, DUMMY - ud, (float)nd);
                        newC[ic + k] = (m == -INFINITY) ? 0.f : m + fpm::fast_log2(sk);
                    }
                }
                __syncthreads();
            }
            for (int k = tid; k < limC; k += 1024) potC[k] = newC[k];
            __syncthreads();
            return;
        }
        if (fast && vec) {
            // thread = (column quad q, row group grp); float4 partial sums, combined over groups
            const int nq = limC >> 2, qpad = (nq + 63) / 64 * 64;
            const int groups4 = qpad >= 1024 ? 1 : 1024 / qpad;
            for (int q0 = 0; q0 < nq; q0 += 1024) {
                const int q = q0 + (groups4 == 1 ? tid : tid % qpad), grp = groups4 == 1 ? 0 : tid / qpad;
                const int ic = 4 * q;
                float4 sh = make_float4(0.f, 0.f, 0.f, 0.f), acc = sh;
                if (q < nq) sh = *(const float4*)&potC[ic];
                if (q < nq && grp < groups4) {
#pragma unroll 8
                    for (int ia = grp; ia < limA; ia += groups4) {
                        const float4 v = *(const float4*)(in + (long)ia * sA + ic);
                        const float pa = potA[ia];
                        acc.x += fpm::fast_exp2(v.x * vscale - pa - sh.x);
                        acc.y += fpm::fast_exp2(v.y * vscale - pa - sh.y);
                        acc.z += fpm::fast_exp2(v.z * vscale - pa - sh.z);
                        acc.w += fpm::fast_exp2(v.w * vscale - pa - sh.w);
                    }
                }
                red4[tid] = acc;
                __syncthreads();
                if (grp == 0 && q < nq) {
                    for (int g = 1; g < groups4; ++g) {
                        const float4 o = red4[tid + g * qpad];
                        acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
                    }
                    const float sv[4] = {acc.x, acc.y, acc.z, acc.w}, hv[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        float sk = sv[k];
                        if (add_dummy) sk += (float)nd * fpm::fast_exp2(DUMMY - ud - hv[k]);
                        if (ok_s(sk)) newC[ic + k] = hv[k] + fpm::fast_log2(sk);
                        else redo_sh = 1;
                    }
                }
                __syncthreads();
            }
        } else if (fast) {
            for (int c0 = 0; c0 < limC; c0 += 1024) {
                const int ic = c0 + (groups == 1 ? tid : tid % cpad), grp = groups == 1 ? 0 : tid / cpad;
                const float sh = ic < limC ? potC[ic] : 0.f;
                float s0 = 0.f, s1 = 0.f;
                if (ic < limC && grp < groups) {
                    int ia = grp;
#pragma unroll 4
                    for (; ia + groups < limA; ia += 2 * groups) {
                        s0 += fpm::fast_exp2(val(ia, ic) - potA[ia] - sh);
                        s1 += fpm::fast_exp2(val(ia + groups, ic) - potA[ia + groups] - sh);
                    }
                    if (ia < limA) s0 += fpm::fast_exp2(val(ia, ic) - potA[ia] - sh);
                }
                float s = s0 + s1;
                red_s[tid] = s;
                __syncthreads();
                if (grp == 0 && ic < limC) {
                    for (int g = 1; g < groups; ++g) s += red_s[tid + g * cpad];
                    if (add_dummy) s += (float)nd * fpm::fast_exp2(DUMMY - ud - sh);
                    if (ok_s(s)) newC[ic] = sh + fpm::fast_log2(s);
                    else redo_sh = 1;
                }
                __syncthreads();
            }
        }
        if (fast) {
            const bool redo = redo_sh != 0;
            __syncthreads();                                  // every thread has read the flag
            if (!redo) {
                for (int k = tid; k < limC; k += 1024) potC[k] = newC[k];
                __syncthreads();
                return;
            }
            if (tid == 0) redo_sh = 0;                        // read again only after the barriers below
        }
        for (int c0 = 0; c0 < limC; c0 += 1024) {
            const int ic = c0 + (groups == 1 ? tid : tid % cpad), grp = groups == 1 ? 0 : tid / cpad;
            float m = -INFINITY, s = 0.f;
            if (ic < limC && grp < groups)
#pragma unroll 8
                for (int ia = grp; ia < limA; ia += groups) lse_push(m, s, val(ia, ic) - potA[ia]);
            red_m[tid] = m;
            red_s[tid] = s;
            __syncthreads();
            if (grp == 0 && ic < limC) {
                for (int g = 1; g < groups; ++g) lse_combine(m, s, red_m[tid + g * cpad], red_s[tid + g * cpad]);
                if (add_dummy) lse_combine(m, s, DUMMY - ud, (float)nd);
                potC[ic] = (m == -INFINITY) ? 0.f : m + fpm::fast_log2(s);
            }
            __syncthreads();
        }
    };
    // ud = lse over the valid algorithmic columns of (DUMMY - v)
    auto update_dummy = [&]() {
        const float* v = u_on_A ? potC : potA;
        const int lim = u_on_A ? limC : limA;
        float m = -INFINITY, s = 0.f;
        for (int k = tid; k < lim; k += 1024) lse_push(m, s, DUMMY - v[k]);
        red_m[tid] = m;
        red_s[tid] = s;
        __syncthreads();
        if (tid == 0) {
            float mm = red_m[0], ss = red_s[0];
            for (int k = 1; k < 1024; ++k) lse_combine(mm, ss, red_m[k], red_s[k]);
            ud_sh = mm + fpm::fast_log2(ss);
        }
        __syncthreads();
    };

    for (int it = 0; it < a.iters; ++it) {
        const bool fast = it > 0 && a.fast;
        if ((it & 1) == 0) {           // row normalisation: update u
            if (u_on_A) along_c(false, fast); else along_a(false, fast);
            if (nd > 0) update_dummy();
        } else {                       // column normalisation: update v
            if (u_on_A) along_a(nd > 0, fast); else along_c(nd > 0, fast);
        }
    }

    if (split && xfail_sh) {                          // a sibling never arrived: fail loudly (NaN)
        for (int k = tid; k < limC; k += 1024) potC[k] = NAN;
        __syncthreads();
    }
    // output rows: this workgroup's a-lines; the last sibling also zeroes the box's padding lines
    const int o_lo = a_lo, o_hi = jj == GP - 1 ? boxA : a_hi;
    float* out = a.out + (long)b * a.out_sb;
    const long oA = a.contig_j ? a.out_si : a.out_sj, oC = a.contig_j ? a.out_sj : a.out_si;
    if (vec && a.rw > 1 && oC == 1 && (oA & 3) == 0 && ((unsigned long)out & 15) == 0 && (boxC & 3) == 0) {
        // 16-B loads and stores along c (limC % 4 == 0 under vec; the box's padding written as 0)
        for (int ia = o_lo + wv; ia < o_hi; ia += 16)
            for (int ic = 4 * lane; ic < boxC; ic += 256) {
                float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
                if (ia < limA && ic < limC) {
                    const float4 v = *(const float4*)(in + (long)ia * sA + ic);
                    const float4 pc = *(const float4*)&potC[ic];
                    const float pa = potA[ia];
                    o = make_float4(fpm::fast_exp2(v.x * vscale - pa - pc.x), fpm::fast_exp2(v.y * vscale - pa - pc.y),
                                    fpm::fast_exp2(v.z * vscale - pa - pc.z), fpm::fast_exp2(v.w * vscale - pa - pc.w));
                }
                *(float4*)(out + ia * oA + ic) = o;
            }
        return;
    }
    for (int ia = o_lo + wv; ia < o_hi; ia += 16)
        for (int ic = lane; ic < boxC; ic += 64) {
            float v = 0.f;
            if (ia < limA && ic < limC) v = fpm::fast_exp2(val(ia, ic) - potA[ia] - potC[ic]);
            out[ia * oA + ic * oC] = v;
        }
}

}  // namespace

// Sinkhorn step form (env FPM_SINKHORN_FAST / fpm_set_tuning("sinkhorn_fast")): 0 max-shifted log
// domain, 1 (default) shifted single-pass lse after the first step; 2 = 1 with scalar loads in the
// streaming kernel.  (A scaling form -- K = exp2(M - pR - pC) absorbed once, later steps as FMA
// row/column rescales with a log-domain fallback when a line sum leaves [2^-40, 2^40] -- was
// measured 2.8x slower at n = 256, tau = 0.01: small temperatures move the potentials by tens of
// log2 units per step, so the guard tripped on most steps; removed.)
// Forward kernel for blocks <= 256 (fpm_set_tuning("sinkhorn_lform")): 1 (default) the L-form
// register kernel, 0 the potential-form sinkhorn_reg_kernel (A/B: 0.444 vs 0.501 ms per launch at
// 1024 pairs, n = 256, 20 steps, profiles/r03k_sinkhorn_kernel_ab.txt; a 512-thread L-form with 128
// entries per thread measured 0.578 ms and was dropped).
int& sinkhorn_lform_flag() {
    static int v = 1;
    return v;
}

// streaming kernel's row step: rows per wave processed together (1 = the single-row loop; A/B)
int& stream_rows_flag() {
    static int v = [] {
        const char* e = getenv("FPM_SK_STREAM_RW");
        return e ? atoi(e) : 4;
    }();
    return v;
}

int& sinkhorn_fast_flag() {
    static int v = [] {
        const char* e = getenv("FPM_SINKHORN_FAST");
        return e ? atoi(e) : 1;
    }();
    return v;
}

// register-tile backward for max(n1max, n2max) <= 256 (called by fpm_sinkhorn_log_bwd; tile:
// B x sinkhorn_reg_tile_elems floats); returns false when the sizes need the general kernel
bool sinkhorn_reg_bwd(const float* s, long s_sb, long s_si, long s_sj, const float* dp, long d_sb, long d_si,
                      long d_sj, float* ds, const int* n1, const int* n2, int B, int n1max, int n2max, int iters,
                      float tau, int dummy_row, float* tile, float* hist, int H, hipStream_t st) {
    const int nmax = n1max > n2max ? n1max : n2max;
    if (nmax > 256 || !(s_sj == 1 || s_si == 1)) return false;
    SinkArgs a = {};
    a.in = s; a.in_sb = s_sb; a.in_si = s_si; a.in_sj = s_sj;
    a.n1 = n1; a.n2 = n2; a.n1max = n1max; a.n2max = n2max;
    a.iters = iters; a.tau = tau; a.dummy_row = dummy_row;
    a.contig_j = (s_sj == 1) ? 1 : 0;
    a.fast = sinkhorn_fast_flag();
    a.dp = dp; a.dp_sb = d_sb; a.dp_si = d_si; a.dp_sj = d_sj;
    a.ds = ds; a.hist = hist; a.H = H; a.ds_tile = tile;
    void (*k)(SinkArgs) = nullptr;
    if (nmax <= 32) k = sinkhorn_reg_kernel<1, 1, true>;
    else if (nmax <= 64) k = sinkhorn_reg_kernel<2, 2, true>;
    else if (nmax <= 128) k = sinkhorn_reg_kernel<4, 4, true>;
    else k = sinkhorn_reg_kernel<8, 8, true>;
    void (*k2)(SinkArgs) = nmax <= 32 ? sinkhorn_bwd_sweep_kernel<1, 1>
                           : nmax <= 64 ? sinkhorn_bwd_sweep_kernel<2, 2>
                           : nmax <= 128 ? sinkhorn_bwd_sweep_kernel<4, 4> : sinkhorn_bwd_sweep_kernel<8, 8>;
    const int er = nmax <= 32 ? 1 : nmax <= 64 ? 2 : nmax <= 128 ? 4 : 8;
    const size_t lds = er >= 8 ? (size_t)(er - er / 2) * er * 1024 * sizeof(float) : 0;   // sweep's dL rows
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)k2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(B), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(k2, dim3(B), dim3(1024), lds, st, a);
    return true;
}

// streaming kernel (boxes over 256): workgroups per pair (FPM_SK_SPLIT, default 2; 1 = one per pair).
// Used only with a caller-provided workspace (fpm_sinkhorn_log_fwd_ws); a pair's result depends on
// this count (the column sums' fp32 summation order), not on the batch it comes in.
int& stream_split_flag() {
    static int v = [] {
        const char* e = getenv("FPM_SK_SPLIT");
        int g = e ? atoi(e) : 2;
        return g < 1 ? 1 : (g > 8 ? 8 : g);
    }();
    return v;
}

// FPM_SK_XACQ=1: the split Sinkhorn's exchange keeps an agent-scope acquire fence after each poll
int& stream_xacq_flag() {
    static int v = [] {
        const char* e = getenv("FPM_SK_XACQ");
        return e ? atoi(e) : 0;
    }();
    return v;
}

namespace {
long sk_cnt_bytes(int B) { return ((long)B * 4 + 15) / 16 * 16; }
long sk_xslot(int n1max, int n2max) { return 2 * (long)((((n1max > n2max ? n1max : n2max) + 3) / 4) * 4); }
}  // namespace

extern "C" long fpm_sinkhorn_ws_bytes(int B, int n1max, int n2max) {
    const int nmax = n1max > n2max ? n1max : n2max;
    const int G = stream_split_flag();
    if (B <= 0 || nmax <= 256 || G <= 1) return 0;
    return sk_cnt_bytes(B) + (long)B * G * 2 * sk_xslot(n1max, n2max) * 4;
}

extern "C" int fpm_sinkhorn_log_fwd_ws(const float* s, long s_sb, long s_si, long s_sj, float* out, long o_sb,
                                       long o_si, long o_sj, const int* n1, const int* n2, int B, int n1max,
                                       int n2max, int iters, float tau, int dummy_row, void* ws, long ws_bytes,
                                       void* stream) {
    FPM_CHECK_ARG(B >= 0 && n1max > 0 && n2max > 0, "sinkhorn: bad sizes");
    FPM_CHECK_ARG(n1max <= SK_MAXN && n2max <= SK_MAXN, "sinkhorn: n1max/n2max > %d not supported (%d,%d)",
                  SK_MAXN, n1max, n2max);
    if (B == 0) return 0;
    SinkArgs a = {};
    a.in = s; a.in_sb = s_sb; a.in_si = s_si; a.in_sj = s_sj;
    a.out = out; a.out_sb = o_sb; a.out_si = o_si; a.out_sj = o_sj;
    a.n1 = n1; a.n2 = n2; a.n1max = n1max; a.n2max = n2max;
    a.iters = iters; a.tau = tau; a.dummy_row = dummy_row;
    a.contig_j = (s_sj == 1) ? 1 : 0;
    a.fast = sinkhorn_fast_flag();
    a.rw = stream_rows_flag();
    a.B = B;
    a.split = 1;
    FPM_CHECK_ARG(s_sj == 1 || s_si == 1, "sinkhorn: one of the input's row/column strides must be 1");
    int nmax = n1max > n2max ? n1max : n2max;
    hipStream_t st = (hipStream_t)stream;
    void (*k)(SinkArgs) = nullptr;
    if (sinkhorn_lform_flag()) {
        if (nmax <= 32) k = sinkhorn_lform_kernel<1, 2, 1024>;
        else if (nmax <= 64) k = sinkhorn_lform_kernel<2, 2, 1024>;
        else if (nmax <= 128) k = sinkhorn_lform_kernel<4, 4, 1024>;
        else if (nmax <= 256) k = sinkhorn_lform_kernel<8, 8, 1024>;
    } else {
        if (nmax <= 32) k = sinkhorn_reg_kernel<1, 1>;
        else if (nmax <= 64) k = sinkhorn_reg_kernel<2, 2>;
        else if (nmax <= 128) k = sinkhorn_reg_kernel<4, 4>;
        else if (nmax <= 256) k = sinkhorn_reg_kernel<8, 8>;
    }
    if (k) {
        hipLaunchKernelGGL(k, dim3(B), dim3(1024), 0, st, a);
        return fpm::check_launch("fpm_sinkhorn_log_fwd");
    }
    const long need = fpm_sinkhorn_ws_bytes(B, n1max, n2max);
    unsigned grid = (unsigned)B;
    if (ws && need > 0) {
        FPM_CHECK_ARG(ws_bytes >= need, "sinkhorn: workspace %ld B < %ld B (fpm_sinkhorn_ws_bytes)", ws_bytes, need);
        FPM_CHECK_ARG(((uintptr_t)ws & 15) == 0, "sinkhorn: workspace not 16-B aligned");
        a.split = stream_split_flag();
        a.xacq = stream_xacq_flag();
        a.xcnt = (int*)ws;
        a.xbuf = (float*)((char*)ws + sk_cnt_bytes(B));
        a.xslot = sk_xslot(n1max, n2max);
        // arrival counters zeroed on the stream before every launch (a memset node under capture)
        FPM_CHECK_ARG(hipMemsetAsync(ws, 0, (size_t)sk_cnt_bytes(B), st) == hipSuccess, "sinkhorn: counter memset failed");
        grid = (unsigned)(((B + 7) / 8) * 8 * a.split);
    }
    hipLaunchKernelGGL(sinkhorn_stream_kernel, dim3(grid), dim3(1024), 0, st, a);
    return fpm::check_launch("fpm_sinkhorn_log_fwd");
}

// Without a workspace the streaming kernel runs one workgroup per pair.
extern "C" int fpm_sinkhorn_log_fwd(const float* s, long s_sb, long s_si, long s_sj, float* out,
                                    long o_sb, long o_si, long o_sj, const int* n1, const int* n2,
                                    int B, int n1max, int n2max, int iters, float tau, int dummy_row,
                                    void* stream) {
    return fpm_sinkhorn_log_fwd_ws(s, s_sb, s_si, s_sj, out, o_sb, o_si, o_sj, n1, n2, B, n1max, n2max, iters, tau,
                                   dummy_row, nullptr, 0, stream);
}
