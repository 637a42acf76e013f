// Two-workgroups-per-CU 256 x 128 bf16 MFMA GEMM tile: the SplineConv (node, cell) product GEMM.
// Same contract and per-element accumulation order as gemm_big_kernel<256> / gemm_phase_kernel (one
// v_mfma_f32_16x16x32_bf16 per 32-deep K step, K ascending), so the outputs are bit-identical.
//
// Why: the 256 x 256 phase kernel holds 135 KB of LDS, so one workgroup owns a CU and its fixed
// per-tile cost -- the prologue's first K-tiles and the epilogue image + 128 KB store, 34 % of a
// K = 768 tile -- leaves the matrix pipes idle.  Here a workgroup needs 72 KB, two
// run on every CU, and while one fills its ring or stores its tile the other's MFMAs run: the
// hardware interleaves the two tiles' phases (a ping-pong without a persistent loop; the grid stays
// one tile per workgroup, so the other pipeline stream's kernels still interleave).
//
// * 256 threads = 4 waves, 2 (rows) x 2 (cols); a wave owns rows {h*128 + wr*64 + [0,64)}, h in {0,1},
//   and columns wc*64 + [0,64): 2 x 4 x 4 16x16 fragments = 32 MFMA per 32-deep K-tile.  Each SIMD
//   carries one wave of each of the CU's two workgroups.
// * BK = 32: an LDS row is 64 B (4 K-chunks of 16 B); chunk c of row r sits in slot
//   PERM[c] ^ ((r >> 2) & 3), PERM = {0, 3, 1, 2}: the 16-lane groups of ds_read_b128 (16 rows at one
//   chunk per quarter-wave) then hit 16 distinct (row mod 4, slot) = bank quads -- conflict-free.
//   The LDS-DMA (global_load_lds, 16 B per lane, 1 KB = 16 rows per wave-instruction) writes lane-
//   linearly, so each lane's SOURCE address carries the inverse permutation (and the row gather).
// * Three-stage ring (24 KB per stage: A 16 KB + B 8 KB): at the top of K-step t every wave retires
//   its own DMA of K-tile t (vmcnt(6): K-tile t + 1's six loads stay in flight), a raw barrier
//   publishes it and certifies that every wave finished reading stage (t - 1) % 3, which then
//   receives K-tile t + 2.
// * Epilogue through LDS (the stages' space): bf16 [256][128] image with 272-B rows, 16-B stores.
#pragma once
#include <type_traits>
#include "gemm_big.h"

namespace fpm {

constexpr int PP_BM = 256, PP_BN = 128, PP_BK = 32, PP_THREADS = 256, PP_NST = 3;
constexpr int PP_A_BYTES = PP_BM * PP_BK * 2;            // 16 KB
constexpr int PP_B_BYTES = PP_BN * PP_BK * 2;            // 8 KB
constexpr int PP_STAGE = PP_A_BYTES + PP_B_BYTES;
constexpr int PP_ROW_OUT = PP_BN * 2 + 16;                // bf16 epilogue row (B)
constexpr int PP_SMEM = g2_max(PP_NST * PP_STAGE, PP_BM * PP_ROW_OUT);
static_assert(PP_SMEM <= 80 * 1024, "two workgroups per CU need <= 80 KB of LDS each");

inline unsigned pp_grid(int N, int mtiles) { return remap_grid_big(N, PP_BN, mtiles); }

__device__ __forceinline__ int pp_slot(int chunk, int row) {
    return ((0x2130 >> (4 * chunk)) & 3) ^ ((row >> 2) & 3);           // PERM = {0, 3, 1, 2}
}
__device__ __forceinline__ int pp_chunk(int slot, int row) {
    return (0x1320 >> (4 * (slot ^ ((row >> 2) & 3)))) & 3;             // PERM^-1 = {0, 2, 3, 1}
}

template <int EPI>
__global__ __launch_bounds__(PP_THREADS, 2) void gemm_pp_kernel(GemmParams p) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[PP_SMEM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int batch = blockIdx.z;

    const int nt = (p.N + PP_BN - 1) / PP_BN;
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
        row0 = mtile * PP_BM;
        row_end = p.M;
    }
    const int n0 = ntile * PP_BN;
    const bf16_t* A = (const bf16_t*)p.A + (long)batch * p.sA;
    const bf16_t* Bg = (const bf16_t*)p.B + (long)batch * p.sB + (long)group * p.sB_seg;

    // DMA sources: A pieces 4w..4w+3 (rows 16 * piece + (lane >> 2)), B pieces 2w, 2w+1; lane slot
    // lane & 3 receives the K-chunk pp_chunk(slot, row)
    const bf16_t* asrc[4];
    const bf16_t* bsrc[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (wave * 4 + i) * 16 + (lane >> 2);
        int gr = row0 + r;
        gr = gr < row_end ? gr : row0;                    // clamp: rows past the end are never stored
        const long arow = p.a_rows ? (long)p.a_rows[gr] : (long)gr;
        asrc[i] = A + arow * p.lda + pp_chunk(lane & 3, r) * 8;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (wave * 2 + i) * 16 + (lane >> 2);
        const int n = n0 + r < p.N ? n0 + r : p.N - 1;    // clamp: columns past N are never stored
        bsrc[i] = Bg + (long)n * p.ldb + pp_chunk(lane & 3, r) * 8;
    }
    auto issue = [&](int stage, int kt) {
        unsigned char* As = smem + stage * PP_STAGE;
        unsigned char* Bs = As + PP_A_BYTES;
        const int k0 = kt * PP_BK;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(asrc[i] + k0), (lds_ptr_t)(As + (wave * 4 + i) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[i] + k0), (lds_ptr_t)(Bs + (wave * 2 + i) * 1024), 16,
                                             0, 0);
    };

    // fragment reads: row R = base + f * 16 + (lane & 15), chunk lane >> 4 at slot pp_slot(chunk, R)
    const int so = pp_slot(lane >> 4, lane & 15) * 16;
    const int a_off = (wr * 64 + (lane & 15)) * 64 + so;
    const int b_off = (wc * 64 + (lane & 15)) * 64 + so;

    f32x4_t acc[2][4][4];                                 // [h][fm][fn]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int stage) __attribute__((always_inline)) {
        const unsigned char* As = smem + stage * PP_STAGE;
        const unsigned char* Bs = As + PP_A_BYTES;
        bf16x8_t a[2][4], b[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) b[f] = *(const bf16x8_t*)(Bs + b_off + f * 1024);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int f = 0; f < 4; ++f) a[h][f] = *(const bf16x8_t*)(As + a_off + h * 8192 + f * 1024);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < 4; ++fn)
                    acc[h][fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][fm], b[fn], acc[h][fm][fn], 0, 0, 0);
    };

    const int ktiles = p.K / PP_BK;                       // >= 1 (K % 64 == 0 checked by the launcher)
    issue(0, 0);
    if (ktiles > 1) issue(1, 1);
    for (int kt = 0; kt < ktiles; ++kt) {
        if (kt + 1 < ktiles) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + 2 < ktiles) issue((kt + 2) % PP_NST, kt + 2);
        compute(kt % PP_NST);
    }
    __syncthreads();                                       // the epilogue reuses the stages' LDS

    int n1b = 0, n2b = 0;
    if (EPI == EPI_AFFINITY) { n1b = p.n1[batch]; n2b = p.n2[batch]; }
    constexpr int ROW = PP_ROW_OUT;
    const int lr = wr * 64 + (lane >> 4) * 4, lc = wc * 64 + (lane & 15);
    auto image = [&](auto hb) __attribute__((always_inline)) {
        constexpr bool HB = decltype(hb)::value;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int wo = (h * 128 + lr) * ROW + lc * 2;
            asm volatile("" : "+v"(wo));                  // a base of its own per half
            unsigned char* wb = smem + wo;
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int j = 0; j < 4; j += 2) {          // rows j, j+1: one v_cvt_pk_bf16_f32
                    const int r = h * 128 + lr + fm * 16 + j;
#pragma unroll
                    for (int fn = 0; fn < 4; ++fn) {
                        const int c = lc + fn * 16;
                        const int n = n0 + c < p.N ? n0 + c : p.N - 1;
                        const uint32_t pk =
                            f2bf2(g2_epi<EPI, HB>(p.bias, acc[h][fm][fn][j], row0 + r, n, n1b, n2b),
                                  g2_epi<EPI, HB>(p.bias, acc[h][fm][fn][j + 1], row0 + r + 1, n, n1b, n2b));
                        const int off = (fm * 16 + j) * ROW + fn * 32;
                        *(bf16_t*)(wb + off) = (bf16_t)pk;
                        *(bf16_t*)(wb + off + ROW) = (bf16_t)(pk >> 16);
                    }
                }
        }
    };
    if (p.bias) image(std::true_type{});
    else image(std::false_type{});
    __syncthreads();
    bf16_t* Ct = (bf16_t*)p.Ct + (long)batch * p.sC;
    constexpr int CH = PP_BN / 8;                          // 16-B chunks per row
    if (p.store_sc1) {
        typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(Ct + (long)row0 * p.ldc + n0), (short)0, (int)(PP_BM * p.ldc * 2), 0x00020000);
#pragma unroll 4
        for (int it = 0; it < PP_BM * CH / PP_THREADS; ++it) {
            const int idx = it * PP_THREADS + tid;
            const int r = idx / CH, ch = idx % CH;
            if (row0 + r < row_end && n0 + ch * 8 < p.N) {
                const uint4 v = *(const uint4*)(smem + r * ROW + ch * 16);
                const u32x4_t pk = {v.x, v.y, v.z, v.w};
                __builtin_amdgcn_raw_buffer_store_b128(pk, rc, (int)((r * p.ldc + ch * 8) * 2), 0, 16);
            }
        }
    } else {
#pragma unroll 4
        for (int it = 0; it < PP_BM * CH / PP_THREADS; ++it) {
            const int idx = it * PP_THREADS + tid;
            const int r = idx / CH, ch = idx % CH;
            if (row0 + r < row_end && n0 + ch * 8 < p.N) {
                const uint4 v = *(const uint4*)(smem + r * ROW + ch * 16);
                *(uint4*)(Ct + (long)(row0 + r) * p.ldc + n0 + ch * 8) = v;
            }
        }
    }
}

// launch policy (product GEMM, bf16 output): FPM_GEMM_PP=1 (fpm_set_tuning("gemm_pp", 1)) picks
// this kernel over the phase kernel; both are bit-identical
int& gemm_pp_flag();
inline bool use_gemm_pp(int K) { return gemm_pp_flag() != 0 && K % 64 == 0 && K >= PP_BK; }

}  // namespace fpm
