// 256-row bf16 MFMA GEMM tiles (256 x 256 and 256 x 128) for the large bf16 GEMMs: the SplineConv
// (node, cell) product GEMM and the AFA-U projections / FFN.
//
//   C[r, n] = epi( sum_k A[row(r), k] * B_g[n, k] (+ bias[n]) )   bf16 operands, fp32 accumulate
//
// * 512 threads = 8 waves; BN = 256: 2 (M) x 4 (N) waves of 128 x 64, BN = 128: 4 x 2 waves of
//   64 x 64, as 16x16x32 MFMA fragments.
// * A and B K-tiles (BK = 64, 128 B per row) are staged global -> LDS with global_load_lds
//   (16 B per lane, no VGPR round trip); the per-lane SOURCE address carries the row gather and an
//   XOR swizzle, the LDS image stays lane-linear: LDS row r, 16-B slot s holds K-chunk
//   s ^ ((r >> 1) & 7).  A fragment read (16 lanes = 16 consecutive rows at one K-chunk) then
//   touches 16 distinct 16-B slots of the 256-B bank row: conflict-free ds_read_b128.
// * Two LDS stages: the loads of K-tile t+1 are issued before the MFMAs of tile t and retired by
//   the barrier that ends step t.
// * Epilogue through LDS (rows padded by 16 B): bf16 output in one pass, fp32 output in two
//   128-row halves; 16-B coalesced global stores; optional bias, then ReLU or the per-pair
//   affinity mask + softplus on the fp32 accumulator.
// * Requirements (checked by the launchers): K % 64 == 0 (callers pad K with zeros), N % 8 == 0,
//   lda/ldb % 8 == 0, ldc 16-B aligned rows.  Rows past M and columns past N are clamped on load
//   and never stored.
// * Tile order: the XCD-chunked remap of gemm_core.h; grouped mode reads a (group, row0) table
//   built for 256-row tiles, group g selecting B + g * sB_seg.
#pragma once
#include <type_traits>
#include "gemm_core.h"

namespace fpm {

constexpr int G2_BM = 256, G2_BK = 64, G2_THREADS = 512;
constexpr int G2_A_BYTES = G2_BM * G2_BK * 2;             // 32 KiB A tile per stage
constexpr int g2_max(int a, int b) { return a > b ? a : b; }

template <int BN> struct G2Cfg {
    static constexpr int WM = BN == 256 ? 2 : 4;          // waves along M
    static constexpr int WN = 8 / WM;                     // waves along N
    static constexpr int FM = G2_BM / WM / 16;            // 16-row fragments per wave
    static constexpr int FN = BN / WN / 16;               // 16-col fragments per wave (4)
    static constexpr int B_BYTES = BN * G2_BK * 2;
    static constexpr int STAGE = G2_A_BYTES + B_BYTES;
    static constexpr int BPIECES = BN / 8 / 8;            // 8-row pieces of B per wave
    // K-tile stages in LDS: 3 for BN = 128 (the DMA of K-tile t + 2 in flight while t computes;
    // 144 KB), 2 for BN = 256 (its 64 KB stages; the phase kernel covers that shape)
    static constexpr int NST = BN == 128 ? 3 : 2;
    static constexpr int LPI = 4 + BPIECES;               // global_load_lds per thread per K-tile
    // stages; bf16 epilogue [256][2BN+16 B]; fp32 epilogue half [128][4BN+16 B]
    static constexpr int SMEM = g2_max(NST * STAGE, g2_max(G2_BM * (2 * BN + 16), 128 * (4 * BN + 16)));
};

inline unsigned remap_grid_big(int N, int BN, int mtiles, int cm = 4) {
    long nt = (N + BN - 1) / BN, chunk = (long)cm * nt;
    long t = nt * mtiles;
    if (mtiles < REMAP_MIN) return (unsigned)t;
    return (unsigned)((t + 8 * chunk - 1) / (8 * chunk) * (8 * chunk));
}
inline unsigned remap_grid256(int N, int mtiles) { return remap_grid_big(N, 256, mtiles); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

// epilogue: optional bias, then store / ReLU / the vertex-affinity mask + softplus (compiled per
// variant so the unrolled 128-element epilogue stays small)
// HB == (bias != nullptr), a compile-time branch of the caller: tested per element, the bias check
// compiled to a scalar branch and two VALU per accumulator (the phase GEMM's epilogue image phase
// 7.4 -> 5.0 K clocks per tile once hoisted, tools/gemm_bench.hip -DGP_PROBE)
template <int EPI, bool HB>
__device__ __forceinline__ float g2_epi(const float* __restrict__ bias, float v, int r, int n, int n1b, int n2b) {
    if (EPI == EPI_NORM_OUT) return v;        // bias and norm already applied to the accumulators
    if (HB) v += bias[n];
    if (EPI == EPI_RELU) return fmaxf(v, 0.f);
    if (EPI == EPI_AFFINITY) return (r < n2b && n < n1b) ? softplus_fast(v) - 0.5f : 0.f;
    return v;
}

template <int BN, int EPI, bool F32OUT>
__global__ __launch_bounds__(G2_THREADS, 1) void gemm_big_kernel(GemmParams p) {
    using Cfg = G2Cfg<BN>;
    constexpr int FM = Cfg::FM, FN = Cfg::FN;
    __shared__ __attribute__((aligned(16))) unsigned char smem[Cfg::SMEM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
    const int batch = blockIdx.z;

    // XCD-chunked tile order (see gemm_core.h)
    const int nt = (p.N + BN - 1) / BN;
    const int q = remap_tile(nt, p.remap_mtiles);
    const int mtile = q / nt, ntile = q - mtile * nt;
    if (mtile >= p.remap_mtiles) return;
    int group = 0, row0, row_end;
    if (p.tile_info) {
        group = p.tile_info[2 * mtile];
        if (group < 0) return;
        row0 = p.tile_info[2 * mtile + 1];
        row_end = p.group_off[group + 1];
    } else {
        row0 = mtile * G2_BM;
        row_end = p.M;
    }
    const int n0 = ntile * BN;
    const bf16_t* A = (const bf16_t*)p.A + (long)batch * p.sA;
    const bf16_t* Bg = (const bf16_t*)p.B + (long)batch * p.sB + (long)group * p.sB_seg;

    // staging: a piece is 8 rows x 128 B; wave w issues A pieces 4w..4w+3 and its share of B.
    // lane: row 8*piece + (lane >> 3), slot lane & 7, K-chunk slot ^ ((row >> 1) & 7)
    const bf16_t* asrc[4];
    const bf16_t* bsrc[Cfg::BPIECES];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (wave * 4 + i) * 8 + (lane >> 3);
        const int kc = (lane & 7) ^ ((r >> 1) & 7);
        int gr = row0 + r;
        gr = gr < row_end ? gr : row0;                    // clamp: rows past the end are never stored
        const long arow = p.a_rows ? (long)p.a_rows[gr] : (long)gr;
        asrc[i] = A + arow * p.lda + kc * 8;
    }
#pragma unroll
    for (int i = 0; i < Cfg::BPIECES; ++i) {
        const int r = (wave * Cfg::BPIECES + i) * 8 + (lane >> 3);
        const int kc = (lane & 7) ^ ((r >> 1) & 7);
        const int n = n0 + r < p.N ? n0 + r : p.N - 1;    // clamp: columns past N are never stored
        bsrc[i] = Bg + (long)n * p.ldb + kc * 8;
    }
    auto issue = [&](int stage, int kt) {
        unsigned char* As = smem + stage * Cfg::STAGE;
        unsigned char* Bs = As + G2_A_BYTES;
        const int k0 = kt * G2_BK;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(asrc[i] + k0), (lds_ptr_t)(As + (wave * 4 + i) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int i = 0; i < Cfg::BPIECES; ++i)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[i] + k0),
                                             (lds_ptr_t)(Bs + (wave * Cfg::BPIECES + i) * 1024), 16, 0, 0);
    };

    // fragment read offsets: row R = base + f*16 + (lane&15), K-chunk c = kk*4 + (lane>>4),
    // slot c ^ ((R>>1)&7) = c ^ ((lane>>1)&7)  (f*16 does not change (R>>1)&7)
    const int xr = (lane >> 1) & 7;
    const int a_base = (wm * FM * 16 + (lane & 15)) * 128;
    const int b_base = (wn * FN * 16 + (lane & 15)) * 128;
    const int s0 = ((lane >> 4) ^ xr) * 16;              // kk = 0
    const int s1 = ((4 + (lane >> 4)) ^ xr) * 16;        // kk = 1

    f32x4_t acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int ktiles = p.K / G2_BK;
    auto compute = [&](int stage) __attribute__((always_inline)) {
        const unsigned char* As = smem + stage * Cfg::STAGE;
        const unsigned char* Bs = As + G2_A_BYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int so = kk ? s1 : s0;
            bf16x8_t a[FM], b[FN];
#pragma unroll
            for (int f = 0; f < FN; ++f) b[f] = *(const bf16x8_t*)(Bs + b_base + f * 2048 + so);
#pragma unroll
            for (int f = 0; f < FM; ++f) a[f] = *(const bf16x8_t*)(As + a_base + f * 2048 + so);
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[fm], b[fn], acc[fm][fn], 0, 0, 0);
        }
    };
    if constexpr (Cfg::NST == 3) {
        // three-stage ring: at the top of step t every wave retires its own DMA of K-tile t (the
        // LPI loads of t + 1 may stay in flight: vmcnt(LPI)), the raw barrier publishes it and
        // certifies that all waves finished reading stage (t - 1) % 3, which then receives K-tile
        // t + 2.  (A __syncthreads() here would drain the in-flight DMA.)  Same per-element
        // accumulation order as the two-stage loop: bit-identical results.
        static_assert(Cfg::LPI == 6, "vmcnt below assumes 6 loads per K-tile (BN = 128)");
        issue(0, 0);
        if (ktiles > 1) issue(1, 1);
        for (int kt = 0; kt < ktiles; ++kt) {
            if (kt + 1 < ktiles) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (kt + 2 < ktiles) issue((kt + 2) % 3, kt + 2);
            compute(kt % 3);
        }
        __syncthreads();                                   // the epilogue reuses the stages' LDS
    } else {
        issue(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int kt = 0; kt < ktiles; ++kt) {
            const int cur = kt & 1;
            if (kt + 1 < ktiles) issue(cur ^ 1, kt + 1);
            compute(cur);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }

    if constexpr (EPI == EPI_NORM_MAX || EPI == EPI_NORM_OUT) {
        // AFA-U instance norms (afau.py:188-199 InstanceNorm1d) over a pair's 256 positions = one
        // 256-row tile, per column c: v = (res +) acc + bias, two-pass mean / variance over the rows
        // (lane column groups via shuffles, the 4 row waves via LDS), y = (v - mean) rstd w + b.
        // NORM_MAX: gmax[pair][c] = max over rows (the block tail); NORM_OUT: y to Cf / Ct through
        // the fp32 store path below (the block head).  Fixed reduction order.
        static_assert(BN == 128 && F32OUT, "norm epilogues: 256 x 128 fp32 tiles");
        float* red = (float*)smem;                         // [WM][BN]; the K loop's LDS is free
        // P = 128 (norm_p): two pairs per tile, each over its WG = WM / 2 row waves; P = 256 is the
        // one-pair form with the same reduction order as before
        const int P = p.norm_p > 0 ? p.norm_p : G2_BM;
        const int WG = Cfg::WM * P / G2_BM;               // row waves per pair
        const int w0 = (wm / WG) * WG;                    // this wave's pair group
        const int pair = (row0 + w0 * FM * 16) / P;
        float v[FM][FN][4];
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                const int c = wn * FN * 16 + fn * 16 + (lane & 15);
                const int n = n0 + c < p.N ? n0 + c : p.N - 1;
                const float bv = p.bias ? p.bias[n] : 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int r = wm * FM * 16 + fm * 16 + (lane >> 4) * 4 + j;
                    // rows past M (the empty second pair of an odd count's last tile): a valid row's
                    // residual instead, their statistics are never written
                    const int gr = row0 + r < p.M ? row0 + r : row0;
                    v[fm][fn][j] = EPI == EPI_NORM_MAX ? p.res[(long)gr * p.ldc + n] + (acc[fm][fn][j] + bv)
                                                       : acc[fm][fn][j] + bv;
                }
            }
        // column reduction over the tile's 256 rows: OP over this lane's rows, the lane groups,
        // then the row waves
        auto colred = [&](float (&t)[FN], bool is_max) {
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                float x = t[fn];
                // lane ^ 16, lane ^ 32 on v_permlane16/32_swap (bit-identical to the shuffle steps)
                x = is_max ? fpm::pair16_max(x) : fpm::pair16_sum(x);
                x = is_max ? fpm::pair32_max(x) : fpm::pair32_sum(x);
                if ((lane >> 4) == 0) red[wm * BN + wn * FN * 16 + fn * 16 + lane] = x;
            }
            __syncthreads();
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                const int c = wn * FN * 16 + fn * 16 + (lane & 15);
                float x = red[w0 * BN + c];
                for (int w = w0 + 1; w < w0 + WG; ++w) x = is_max ? fmaxf(x, red[w * BN + c]) : x + red[w * BN + c];
                t[fn] = x;
            }
            __syncthreads();
        };
        float mean[FN], var[FN];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
            float s = 0.f;
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                for (int j = 0; j < 4; ++j) s += v[fm][fn][j];
            mean[fn] = s;
        }
        colred(mean, false);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
            mean[fn] /= (float)P;
            float s = 0.f;
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float d = v[fm][fn][j] - mean[fn];
                    s += d * d;
                }
            var[fn] = s;
        }
        colred(var, false);
        if constexpr (EPI == EPI_NORM_MAX) {
            float mx[FN];
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                const int c = wn * FN * 16 + fn * 16 + (lane & 15);
                const int n = n0 + c < p.N ? n0 + c : p.N - 1;
                const float rstd = 1.f / sqrtf(var[fn] / (float)P + p.eps);
                const float ww = p.nw[n], bb = p.nb[n];
                float m = -INFINITY;
#pragma unroll
                for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                    for (int j = 0; j < 4; ++j) m = fmaxf(m, (v[fm][fn][j] - mean[fn]) * rstd * ww + bb);
                mx[fn] = m;
            }
            colred(mx, true);
            if (wm == w0 && (lane >> 4) == 0 && pair < p.M / P) {   // (an odd pair count's empty half: no write)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn) {
                    const int c = wn * FN * 16 + fn * 16 + lane;
                    if (n0 + c < p.N) p.gmax[(long)pair * p.N + n0 + c] = mx[fn];
                }
            }
            return;
        } else {
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                const int c = wn * FN * 16 + fn * 16 + (lane & 15);
                const int n = n0 + c < p.N ? n0 + c : p.N - 1;
                const float rstd = 1.f / sqrtf(var[fn] / (float)P + p.eps);
                const float ww = p.nw[n], bb = p.nb[n];
#pragma unroll
                for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[fm][fn][j] = (v[fm][fn][j] - mean[fn]) * rstd * ww + bb;
            }
        }
    }
    // epilogue through LDS
    int n1b = 0, n2b = 0;
    if (EPI == EPI_AFFINITY) { n1b = p.n1[batch]; n2b = p.n2[batch]; }
    if (!F32OUT) {
        // bf16 tile [256][BN] with (2*BN + 16)-B rows
        constexpr int ROW = BN * 2 + 16;
        // rows j, j+1 of a lane's column converted by one v_cvt_pk_bf16_f32, the halves stored
        // with ds_write_b16 / ds_write_b16_d16_hi
        auto image = [&](auto hb) __attribute__((always_inline)) {
            constexpr bool HB = decltype(hb)::value;
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                for (int j = 0; j < 4; j += 2) {
                    const int r = wm * FM * 16 + fm * 16 + (lane >> 4) * 4 + j;
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn) {
                        const int c = wn * FN * 16 + fn * 16 + (lane & 15);
                        const int n = n0 + c < p.N ? n0 + c : p.N - 1;
                        const uint32_t pk = f2bf2(g2_epi<EPI, HB>(p.bias, acc[fm][fn][j], row0 + r, n, n1b, n2b),
                                                  g2_epi<EPI, HB>(p.bias, acc[fm][fn][j + 1], row0 + r + 1, n, n1b, n2b));
                        *(bf16_t*)(smem + r * ROW + c * 2) = (bf16_t)pk;
                        *(bf16_t*)(smem + (r + 1) * ROW + c * 2) = (bf16_t)(pk >> 16);
                    }
                }
        };
        if (p.bias) image(std::true_type{});
        else image(std::false_type{});
        __syncthreads();
        bf16_t* Ct = (bf16_t*)p.Ct + (long)batch * p.sC;
        constexpr int CH = BN / 8;                        // 16-B chunks per row
#pragma unroll 4
        for (int it = 0; it < G2_BM * CH / G2_THREADS; ++it) {
            const int idx = it * G2_THREADS + tid;
            const int r = idx / CH, ch = idx % CH;
            if (row0 + r < row_end && n0 + ch * 8 < p.N) {
                uint4 v = *(const uint4*)(smem + r * ROW + ch * 16);
                *(uint4*)(Ct + (long)(row0 + r) * p.ldc + n0 + ch * 8) = v;
            }
        }
    } else {
        // fp32 tile in two 128-row halves, [128][BN] with (4*BN + 16)-B rows
        constexpr int ROW = BN * 4 + 16;
        constexpr int WAVES_PER_HALF_M = Cfg::WM / 2;     // waves along M in each half
        float* Cf = p.Cf ? p.Cf + (long)batch * p.sC : nullptr;
        constexpr int CH = BN / 4;
        for (int h = 0; h < 2; ++h) {
            if (wm / WAVES_PER_HALF_M == h) {
                auto image = [&](auto hb) __attribute__((always_inline)) {
                    constexpr bool HB = decltype(hb)::value;
#pragma unroll
                    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int r = wm * FM * 16 + fm * 16 + (lane >> 4) * 4 + j;   // tile row
#pragma unroll
                            for (int fn = 0; fn < FN; ++fn) {
                                const int c = wn * FN * 16 + fn * 16 + (lane & 15);
                                const int n = n0 + c < p.N ? n0 + c : p.N - 1;
                                *(float*)(smem + (r - h * 128) * ROW + c * 4) =
                                    g2_epi<EPI, HB>(p.bias, acc[fm][fn][j], row0 + r, n, n1b, n2b);
                            }
                        }
                };
                if (p.bias) image(std::true_type{});
                else image(std::false_type{});
            }
            __syncthreads();
            // the bf16 operand copy beside (or, Cf null, instead of) the fp32 rows: plain (NORM_OUT)
            // or split [hi | lo | hi] (p.split), K padding columns [N, segment) written as zeros
            const bool copy = p.Ct && (EPI == EPI_NORM_OUT || p.split > 0);
            const long seg = p.split > 0 ? p.split : p.ldt;
#pragma unroll 4
            for (int it = 0; it < 128 * CH / G2_THREADS; ++it) {
                const int idx = it * G2_THREADS + tid;
                const int r = idx / CH, ch = idx % CH;
                const int gr = row0 + h * 128 + r;
                const int col = n0 + ch * 4;
                if (gr < row_end && col < p.N) {
                    uint4 v = *(const uint4*)(smem + r * ROW + ch * 16);
                    if (Cf) *(uint4*)(Cf + (long)gr * p.ldc + col) = v;
                    if (copy) {
                        bf16_t* ct = (bf16_t*)p.Ct + (long)gr * p.ldt + col;
                        uint2 o;
                        o.x = f2bf2(__uint_as_float(v.x), __uint_as_float(v.y));
                        o.y = f2bf2(__uint_as_float(v.z), __uint_as_float(v.w));
                        *(uint2*)ct = o;
                        if (p.split > 0) {
                            // lo = bf16(v - float(hi)): hi + lo carries ~16 mantissa bits of v
                            uint2 l;
                            l.x = f2bf2(__uint_as_float(v.x) - __uint_as_float(o.x << 16),
                                        __uint_as_float(v.y) - __uint_as_float(o.x & 0xffff0000u));
                            l.y = f2bf2(__uint_as_float(v.z) - __uint_as_float(o.y << 16),
                                        __uint_as_float(v.w) - __uint_as_float(o.y & 0xffff0000u));
                            *(uint2*)(ct + p.split) = l;
                            *(uint2*)(ct + 2 * p.split) = o;
                        }
                    }
                } else if (copy && gr < row_end && col < seg) {
                    bf16_t* ct = (bf16_t*)p.Ct + (long)gr * p.ldt + col;                     // K padding
                    *(uint2*)ct = make_uint2(0u, 0u);
                    if (p.split > 0) {
                        *(uint2*)(ct + p.split) = make_uint2(0u, 0u);
                        *(uint2*)(ct + 2 * p.split) = make_uint2(0u, 0u);
                    }
                }
            }
            __syncthreads();
        }
    }
}

}  // namespace fpm
