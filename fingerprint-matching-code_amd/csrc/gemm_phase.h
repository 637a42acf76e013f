// Phase-pipelined 256 x 256 bf16 MFMA GEMM tile (the SplineConv (node, cell) product GEMM and the
// other large bf16 GEMMs with N % 256 == 0).  Same contract and results as gemm_big_kernel<256>
// (gemm_big.h): identical per-element accumulation order, so the outputs are bit-identical.
//
// Why a second kernel: gemm_big_kernel retires every K-tile's LDS-DMA with vmcnt(0) + a workgroup
// barrier, so each K-step stalls on its own prefetch (the "~900 TF" structure).  Here the K loop is
// cut into PHASES, one per C-quadrant of each wave, and the LDS-DMA stream runs 3-4 phases ahead:
//
// * 512 threads = 8 waves = 2 groups (wr) x 4 (wc).  A wave owns rows {h*128 + wr*64 + [0,64)} and
//   columns {g*128 + wc*32 + [0,32)}, h, g in {0,1}: its 128 x 64 output is four 64 x 32 quadrants
//   (h, g), each 4 x 2 16x16 fragments = 16 MFMA 16x16x32 per 64-deep K-tile.
// * LDS: two K-tile buffers, each four HALF-TILES A0, A1 (A rows h*128..+128), B0, B1 (B rows =
//   output columns g*128..+128); a half-tile is 128 rows x 128 B (BK = 64 bf16), filled by two
//   global_load_lds_dwordx4 per thread, XOR-swizzled on the source address exactly as gemm_big.h.
// * K-tile t runs phases q = 0..3 on quadrants (0,0) (0,1) (1,1) (1,0); the A fragments of half h
//   and the B fragments of both halves stay in registers across the phases that share them, so
//   each K-tile reads the 24 fragments once: q0 reads A0 + B0, q1 B1, q2 A1, q3 nothing.
// * One half-tile of LDS-DMA is issued per phase, in the order A0 B0 B1 A1 of each K-tile, six
//   half-tiles ahead of the phase stream: phase phi issues half-tile j = phi + 6 and, before that,
//   retires j = phi + 2 with s_waitcnt vmcnt(6) (2 instructions per younger half-tile).  Every
//   half-tile is retired at least one phase before its first read and re-staged at least two
//   phases after its last read (the RAW / WAR rules with the barriers below).
// * Each phase: [wait; issue; ds_reads] s_barrier, lgkmcnt(0), MFMAs at raised priority, s_barrier.
//   Group wr = 1 runs one barrier behind group 0, so on every SIMD one wave's MFMAs overlap the
//   other wave's LDS reads and DMA issue.  Raw s_barrier only: __syncthreads() would drain the
//   in-flight DMA (vmcnt(0)).  All LDS is the one __shared__ array (a second one makes the
//   compiler wait vmcnt(0) before the ds_reads).
// * The last two K-tiles are peeled with their exact vmcnt counts (no issues past the end).
#pragma once
#include <type_traits>
#include "gemm_big.h"

namespace fpm {

constexpr int GP_HALF = 128 * 128;                        // bytes per half-tile
constexpr int GP_SMEM = g2_max(8 * GP_HALF, G2_BM * (2 * 256 + 16));
constexpr int GP_MIN_KTILES = 2;

#define FPM_VMCNT(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")

// GP_PROBE (tools/gemm_bench.hip only, never in the library): per-workgroup shader-clock stamps at
// entry, main-loop start, main-loop end, epilogue image written, stores issued, stores retired
// (wave 0) -> gp_probe_buf[wg * 8 + k]
#ifdef GP_PROBE
__device__ unsigned long long* gp_probe_buf;
#define GP_STAMP(k)                                                                                   \
    do {                                                                                              \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                   \
        if (threadIdx.x == 0 && gp_probe_buf)                                                         \
            gp_probe_buf[((long)blockIdx.z * gridDim.x + blockIdx.x) * 8 + (k)] = t_;                   \
    } while (0)
#else
#define GP_STAMP(k)
#endif

#ifndef GP_STAGGER
#define GP_STAGGER 1
#endif
#ifndef GP_PRIO
#define GP_PRIO 1
#endif
// DIRECT (bf16 output): the MFMAs run with swapped operands (weights as the first), so each lane's
// accumulator holds 4 consecutive OUTPUT COLUMNS of one row, and the epilogue stores them straight
// from registers (8 B per lane, no LDS image, no barrier)
template <int EPI, bool F32OUT, bool DIRECT = false>
__global__ __launch_bounds__(G2_THREADS, 1) void gemm_phase_kernel(GemmParams p) {
    constexpr int BN = 256;
    __shared__ __attribute__((aligned(16))) unsigned char smem[GP_SMEM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int batch = blockIdx.z;

    const int nt = (p.N + BN - 1) / BN;
    const int q = remap_tile(nt, p.remap_mtiles, p.remap_cm > 0 ? p.remap_cm : 4);
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

    // DMA sources: half-tile piece i of wave w = rows 8*(2w+i) + (lane>>3) of the half,
    // K-chunk (lane&7) ^ ((row>>1)&7)
    const bf16_t* src[4][2];                              // [A0, A1, B0, B1][piece]
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (wave * 2 + i) * 8 + (lane >> 3);
        const int kc = (lane & 7) ^ ((r >> 1) & 7);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int gr = row0 + h * 128 + r;
            gr = gr < row_end ? gr : row0;                // clamp: rows past the end are never stored
            const long arow = p.a_rows ? (long)p.a_rows[gr] : (long)gr;
            src[h][i] = A + arow * p.lda + kc * 8;
            const int n = n0 + h * 128 + r < p.N ? n0 + h * 128 + r : p.N - 1;
            src[2 + h][i] = Bg + (long)n * p.ldb + kc * 8;
        }
    }
    // half-tile stream j: K-tile j >> 2, kind j & 3 in the order A0 B0 B1 A1 -> buffer slot
    auto issue = [&](int j, int slot) {
        const int t = j >> 2;
        unsigned char* dst = smem + ((t & 1) * 4 + slot) * GP_HALF + wave * 2048;
        const int k0 = t * G2_BK;
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src[slot][0] + k0), (lds_ptr_t)dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src[slot][1] + k0), (lds_ptr_t)(dst + 1024), 16, 0, 0);
    };

    // fragment reads: A half row wr*64 + f*16 + (lane&15) (f < 4), B half row wc*32 + f*16 +
    // (lane&15) (f < 2); K-chunk c = kk*4 + (lane>>4) at slot c ^ ((lane>>1)&7)
    const int xr = (lane >> 1) & 7;
    const int a_off = (wr * 64 + (lane & 15)) * 128;
    const int b_off = (wc * 32 + (lane & 15)) * 128;
    const int s0 = ((lane >> 4) ^ xr) * 16, s1 = ((4 + (lane >> 4)) ^ xr) * 16;

    f32x4_t acc[2][2][4][2];                              // [h][g][fm][fn]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[h][g][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    bf16x8_t a[2][4], b0[2][2], b1[2][2];                 // [kk][frag]

    auto read_a = [&](int t, int h) {
        const unsigned char* base = smem + ((t & 1) * 4 + h) * GP_HALF + a_off;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            a[0][f] = *(const bf16x8_t*)(base + f * 2048 + s0);
            a[1][f] = *(const bf16x8_t*)(base + f * 2048 + s1);
        }
    };
    auto read_b = [&](int t, int g, bf16x8_t (&bb)[2][2]) {
        const unsigned char* base = smem + ((t & 1) * 4 + 2 + g) * GP_HALF + b_off;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            bb[0][f] = *(const bf16x8_t*)(base + f * 2048 + s0);
            bb[1][f] = *(const bf16x8_t*)(base + f * 2048 + s1);
        }
    };
    auto mfma = [&](f32x4_t (&c)[4][2], bf16x8_t (&bb)[2][2]) {
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (GP_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < 2; ++fn) {
                    if constexpr (DIRECT)
                        c[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[kk][fn], a[kk][fm], c[fm][fn], 0, 0, 0);
                    else
                        c[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][fm], bb[kk][fn], c[fm][fn], 0, 0, 0);
                }
        if (GP_PRIO) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
    };
    // slots of the kinds A0 B0 B1 A1
    constexpr int SLOT[4] = {0, 2, 3, 1};
    // one K-tile = 4 phases; VMq = vmcnt before phase q's issue (-1: none), ISSq: phase q issues
    auto ktile = [&](int t, auto VM0, auto VM1, auto VM2, auto VM3, bool iss0, bool iss1, bool iss2, bool iss3) {
        const int phi = 4 * t;
        // q0: quadrant (0,0), reads A0 + B0; issues j = phi + 6 (B1 of t+1)
        if constexpr (decltype(VM0)::value == 6) FPM_VMCNT(6);
        else if constexpr (decltype(VM0)::value == 4) FPM_VMCNT(4);
        else if constexpr (decltype(VM0)::value == 2) FPM_VMCNT(2);
        else if constexpr (decltype(VM0)::value == 0) FPM_VMCNT(0);
        if (iss0) issue(phi + 6, SLOT[(0 + 6) & 3]);
        read_a(t, 0);
        read_b(t, 0, b0);
        mfma(acc[0][0], b0);
        // q1: quadrant (0,1), reads B1; issues A1 of t+1
        if constexpr (decltype(VM1)::value == 6) FPM_VMCNT(6);
        else if constexpr (decltype(VM1)::value == 4) FPM_VMCNT(4);
        else if constexpr (decltype(VM1)::value == 2) FPM_VMCNT(2);
        else if constexpr (decltype(VM1)::value == 0) FPM_VMCNT(0);
        if (iss1) issue(phi + 7, SLOT[(1 + 6) & 3]);
        read_b(t, 1, b1);
        mfma(acc[0][1], b1);
        // q2: quadrant (1,1), reads A1; issues A0 of t+2
        if constexpr (decltype(VM2)::value == 6) FPM_VMCNT(6);
        else if constexpr (decltype(VM2)::value == 4) FPM_VMCNT(4);
        else if constexpr (decltype(VM2)::value == 2) FPM_VMCNT(2);
        else if constexpr (decltype(VM2)::value == 0) FPM_VMCNT(0);
        if (iss2) issue(phi + 8, SLOT[(2 + 6) & 3]);
        read_a(t, 1);
        mfma(acc[1][1], b1);
        // q3: quadrant (1,0), no reads; issues B0 of t+2
        if constexpr (decltype(VM3)::value == 6) FPM_VMCNT(6);
        else if constexpr (decltype(VM3)::value == 4) FPM_VMCNT(4);
        else if constexpr (decltype(VM3)::value == 2) FPM_VMCNT(2);
        else if constexpr (decltype(VM3)::value == 0) FPM_VMCNT(0);
        if (iss3) issue(phi + 9, SLOT[(3 + 6) & 3]);
        mfma(acc[1][0], b0);
    };
    using V6 = std::integral_constant<int, 6>;
    using V4 = std::integral_constant<int, 4>;
    using V2 = std::integral_constant<int, 2>;
    using V0 = std::integral_constant<int, 0>;
    using VN = std::integral_constant<int, -1>;

    GP_STAMP(0);
    const int ktiles = p.K / G2_BK;                       // >= GP_MIN_KTILES (checked by the launcher)
    // prologue: half-tiles j = 0..5 (all of K-tile 0, A0 B0 of K-tile 1); A0(0) B0(0) readable first
#pragma unroll
    for (int j = 0; j < 6; ++j) issue(j, SLOT[j & 3]);
    FPM_VMCNT(8);
    __builtin_amdgcn_s_barrier();
    GP_STAMP(1);
    if (GP_STAGGER && wr == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one barrier behind

    // steady state: phase phi retires j = phi + 2 (vmcnt 6) and issues j = phi + 6
    int t = 0;
    for (; t < ktiles - 2; ++t) ktile(t, V6{}, V6{}, V6{}, V6{}, true, true, true, true);
    // K-tile ktiles-2: issues the last two half-tiles (B1, A1 of the last K-tile)
    ktile(t, V6{}, V6{}, V6{}, V4{}, true, true, false, false);
    // last K-tile: retire j = J-2 (vmcnt 2), J-1 (vmcnt 0), then nothing in flight
    ktile(t + 1, V2{}, V0{}, VN{}, VN{}, false, false, false, false);
    if (GP_STAGGER && wr == 0) __builtin_amdgcn_s_barrier();   // re-align the groups
    __syncthreads();
    GP_STAMP(2);

    // epilogue through LDS (same images as gemm_big_kernel<256>)
    int n1b = 0, n2b = 0;
    if (EPI == EPI_AFFINITY) { n1b = p.n1[batch]; n2b = p.n2[batch]; }
    if constexpr (DIRECT) {
        static_assert(!F32OUT && EPI == EPI_STORE, "DIRECT: bf16 output, plain store");
        // lane: output row  h*128 + wr*64 + fm*16 + (lane & 15), columns g*128 + wc*32 + fn*16 + 4*(lane >> 4) + [0, 4)
        bf16_t* Ct = (bf16_t*)p.Ct + (long)batch * p.sC;
        const int cl = wc * 32 + 4 * (lane >> 4);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) {
                const int r = row0 + h * 128 + wr * 64 + fm * 16 + (lane & 15);
                if (r >= row_end) continue;
                bf16_t* rowp = Ct + (long)r * p.ldc + n0;
#pragma unroll
                for (int g = 0; g < 2; ++g)
#pragma unroll
                    for (int fn = 0; fn < 2; ++fn) {
                        const int c = g * 128 + cl + fn * 16;
                        if (n0 + c >= p.N) continue;
                        const f32x4_t v = acc[h][g][fm][fn];
                        uint2 o;
                        o.x = f2bf2(v[0], v[1]);
                        o.y = f2bf2(v[2], v[3]);
                        *(uint2*)(rowp + c) = o;
                    }
            }
        return;
    }
    if (!F32OUT) {
        constexpr int ROW = BN * 2 + 16;
        // the bias test hoisted out of the image loop (a compile-time branch each; g2_epi)
        // per-lane base of the image (one per 128-row half, so each write's remaining offset is a
        // compile-time constant within the 16-bit LDS offset field)
        const int lr = wr * 64 + (lane >> 4) * 4, lc = wc * 32 + (lane & 15);
        auto image = [&](auto hb) __attribute__((always_inline)) {
            constexpr bool HB = decltype(hb)::value;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int wo = (h * 128 + lr) * ROW + lc * 2;
                asm volatile("" : "+v"(wo));        // a base of its own (not h = 0's + a 17-bit constant)
                unsigned char* wb = smem + wo;
#pragma unroll
                for (int g = 0; g < 2; ++g)
#pragma unroll
                    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                        for (int j = 0; j < 4; j += 2) {     // rows j, j+1: one v_cvt_pk_bf16_f32
                            const int r = h * 128 + lr + fm * 16 + j;
#pragma unroll
                            for (int fn = 0; fn < 2; ++fn) {
                                const int c = g * 128 + lc + fn * 16;
                                const int n = n0 + c < p.N ? n0 + c : p.N - 1;
                                const uint32_t pk =
                                    f2bf2(g2_epi<EPI, HB>(p.bias, acc[h][g][fm][fn][j], row0 + r, n, n1b, n2b),
                                          g2_epi<EPI, HB>(p.bias, acc[h][g][fm][fn][j + 1], row0 + r + 1, n, n1b, n2b));
                                const int off = (fm * 16 + j) * ROW + (g * 128 + fn * 16) * 2;
                                *(bf16_t*)(wb + off) = (bf16_t)pk;
                                *(bf16_t*)(wb + off + ROW) = (bf16_t)(pk >> 16);
                            }
                        }
            }
        };
        if (p.bias) image(std::true_type{});
        else image(std::false_type{});
        __syncthreads();
        GP_STAMP(3);
        bf16_t* Ct = (bf16_t*)p.Ct + (long)batch * p.sC;
        constexpr int CH = BN / 8;
        if (p.store_sc1) {
            // the tile's rows as one buffer resource (256 rows x ldc bf16 < 2 GiB), sc1 stores
            typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
            const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(Ct + (long)row0 * p.ldc + n0), (short)0, (int)(G2_BM * p.ldc * 2), 0x00020000);
#pragma unroll 4
            for (int it = 0; it < G2_BM * CH / G2_THREADS; ++it) {
                const int idx = it * G2_THREADS + tid;
                const int r = idx / CH, ch = idx % CH;
                if (row0 + r < row_end && n0 + ch * 8 < p.N) {
                    const uint4 v = *(const uint4*)(smem + r * ROW + ch * 16);
                    const u32x4_t pk = {v.x, v.y, v.z, v.w};
                    __builtin_amdgcn_raw_buffer_store_b128(pk, rc, (int)((r * p.ldc + ch * 8) * 2), 0, 16);
                }
            }
        } else {
#pragma unroll 4
            for (int it = 0; it < G2_BM * CH / G2_THREADS; ++it) {
                const int idx = it * G2_THREADS + tid;
                const int r = idx / CH, ch = idx % CH;
                if (row0 + r < row_end && n0 + ch * 8 < p.N) {
                    uint4 v = *(const uint4*)(smem + r * ROW + ch * 16);
                    *(uint4*)(Ct + (long)(row0 + r) * p.ldc + n0 + ch * 8) = v;
                }
            }
        }
        GP_STAMP(4);
#ifdef GP_PROBE
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the probe's last stamp: stores retired
        GP_STAMP(5);
#endif
    } else {
        constexpr int ROW = BN * 4 + 16;
        float* Cf = p.Cf + (long)batch * p.sC;
        constexpr int CH = BN / 4;
        auto image = [&](int h, auto hb) __attribute__((always_inline)) {
            constexpr bool HB = decltype(hb)::value;
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = wr * 64 + fm * 16 + (lane >> 4) * 4 + j;     // row within half h
#pragma unroll
                        for (int fn = 0; fn < 2; ++fn) {
                            const int c = g * 128 + wc * 32 + fn * 16 + (lane & 15);
                            const int n = n0 + c < p.N ? n0 + c : p.N - 1;
                            *(float*)(smem + r * ROW + c * 4) =
                                g2_epi<EPI, HB>(p.bias, acc[h][g][fm][fn][j], row0 + h * 128 + r, n, n1b, n2b);
                        }
                    }
        };
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (p.bias) image(h, std::true_type{});
            else image(h, std::false_type{});
            __syncthreads();
#pragma unroll 4
            for (int it = 0; it < 128 * CH / G2_THREADS; ++it) {
                const int idx = it * G2_THREADS + tid;
                const int r = idx / CH, ch = idx % CH;
                const int gr = row0 + h * 128 + r;
                if (gr < row_end && n0 + ch * 4 < p.N) {
                    uint4 v = *(const uint4*)(smem + r * ROW + ch * 16);
                    *(uint4*)(Cf + (long)gr * p.ldc + n0 + ch * 4) = v;
                }
            }
            __syncthreads();
        }
    }
}

#undef FPM_VMCNT

// launch policy: the phase kernel for 256-wide tiles with >= 2 K-tiles; FPM_GEMM_PHASE=0 (or
// fpm_set_gemm_phase(0)) keeps gemm_big_kernel<256> -- an A/B switch, both are bit-identical
int& gemm_phase_flag();
inline bool use_gemm_phase(int K) { return gemm_phase_flag() != 0 && K / G2_BK >= GP_MIN_KTILES; }

}  // namespace fpm
