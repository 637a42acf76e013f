// 256 x 256 bf16 MFMA GEMM tile for the large product GEMM of SplineConv (and any bf16 GEMM with
// N % 256 == 0, K % 64 == 0):
//
//   C[r, n] = sum_k A[row(r), k] * B_g[n, k]        (bf16 operands, fp32 accumulate, bf16 out)
//
// * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns 128 x 64 = 8 x 4 MFMA 16x16x32 tiles.
// * A and B K-tiles (BK = 64, 128 B per row) are staged global -> LDS with global_load_lds
//   (16 B per lane, no VGPR round trip); the per-lane SOURCE address carries the row gather and an
//   XOR swizzle, the LDS image stays lane-linear: LDS row r, 16-B slot s holds K-chunk
//   s ^ ((r >> 1) & 7).  A fragment read (16 lanes = 16 consecutive rows at one K-chunk) then
//   touches 16 distinct 16-B slots of the 256-B bank row: conflict-free ds_read_b128.
// * Two LDS stages: the loads of K-tile t+1 are issued before the MFMAs of tile t and retired by
//   the barrier that ends step t.
// * Epilogue: accumulators -> bf16 -> LDS (rows padded to 528 B) -> 16-B coalesced global stores.
// * Tile order: the XCD-chunked remap of gemm_core.h; grouped mode reads a (group, row0) table
//   built for 256-row tiles, group g selecting B + g * sB_seg.
#pragma once
#include "gemm_core.h"

namespace fpm {

constexpr int G2_BM = 256, G2_BN = 256, G2_BK = 64, G2_THREADS = 512;
constexpr int G2_TILE_BYTES = G2_BM * G2_BK * 2;          // 32 KiB per operand per stage
constexpr int G2_EPI_ROW = G2_BN * 2 + 16;                // padded epilogue row (bytes)
constexpr int G2_SMEM = G2_BM * G2_EPI_ROW;               // 135168 B >= 4 staging tiles (131072 B)

inline unsigned remap_grid256(int N, int mtiles) {
    long nt = N / G2_BN, chunk = 4 * nt;
    long t = nt * mtiles;
    return (unsigned)((t + 8 * chunk - 1) / (8 * chunk) * (8 * chunk));
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

__global__ __launch_bounds__(G2_THREADS, 1) void gemm256_bf16_kernel(GemmParams p) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[G2_SMEM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;

    // XCD-chunked tile order (see gemm_core.h)
    const int nt = p.N / G2_BN;
    const int chunk = 4 * nt;
    const int bi = blockIdx.x >> 3;
    const int q = ((bi / chunk) * 8 + (blockIdx.x & 7)) * chunk + (bi % chunk);
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
    const int n0 = ntile * G2_BN;
    const bf16_t* A = (const bf16_t*)p.A;
    const bf16_t* Bg = (const bf16_t*)p.B + (long)group * p.sB_seg;

    // staging: wave w issues pieces ci = 4w + i (i < 4) of each operand; a piece is 8 rows x 128 B.
    // lane: row 8 ci + (lane >> 3), slot lane & 7, K-chunk slot ^ ((row >> 1) & 7)
    const bf16_t* asrc[4];
    const bf16_t* bsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int ci = wave * 4 + i;
        const int r = ci * 8 + (lane >> 3);
        const int kc = (lane & 7) ^ ((r >> 1) & 7);
        int gr = row0 + r;
        gr = gr < row_end ? gr : row0;                    // clamp: rows past the end are never stored
        const long arow = p.a_rows ? (long)p.a_rows[gr] : (long)gr;
        asrc[i] = A + arow * p.lda + kc * 8;
        bsrc[i] = Bg + (long)(n0 + r) * p.ldb + kc * 8;
    }
    auto issue = [&](int stage, int kt) {
        unsigned char* As = smem + stage * 2 * G2_TILE_BYTES;
        unsigned char* Bs = As + G2_TILE_BYTES;
        const int k0 = kt * G2_BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ci = wave * 4 + i;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(asrc[i] + k0), (lds_ptr_t)(As + ci * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[i] + k0), (lds_ptr_t)(Bs + ci * 1024), 16, 0, 0);
        }
    };

    // fragment read offsets: row R = base + f*16 + (lane&15), K-chunk c = kk*4 + (lane>>4),
    // slot c ^ ((R>>1)&7) = c ^ ((lane>>1)&7)  (f*16 does not change (R>>1)&7)
    const int xr = (lane >> 1) & 7;
    const int a_base = (wm * 128 + (lane & 15)) * 128;
    const int b_base = (wn * 64 + (lane & 15)) * 128;
    const int s0 = (((lane >> 4)) ^ xr) * 16;            // kk = 0
    const int s1 = ((4 + (lane >> 4)) ^ xr) * 16;        // kk = 1

    f32x4_t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int ktiles = p.K / G2_BK;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < ktiles; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < ktiles) issue(cur ^ 1, kt + 1);
        const unsigned char* As = smem + cur * 2 * G2_TILE_BYTES;
        const unsigned char* Bs = As + G2_TILE_BYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int so = kk ? s1 : s0;
            bf16x8_t a[8], b[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) b[f] = *(const bf16x8_t*)(Bs + b_base + f * 2048 + so);
#pragma unroll
            for (int f = 0; f < 8; ++f) a[f] = *(const bf16x8_t*)(As + a_base + f * 2048 + so);
#pragma unroll
            for (int fm = 0; fm < 8; ++fm)
#pragma unroll
                for (int fn = 0; fn < 4; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[fm], b[fn], acc[fm][fn], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // epilogue through LDS: bf16 tile [256][256] with 528-B rows
#pragma unroll
    for (int fm = 0; fm < 8; ++fm)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = wm * 128 + fm * 16 + (lane >> 4) * 4 + j;
#pragma unroll
            for (int fn = 0; fn < 4; ++fn) {
                const int c = wn * 64 + fn * 16 + (lane & 15);
                *(bf16_t*)(smem + r * G2_EPI_ROW + c * 2) = f2bf(acc[fm][fn][j]);
            }
        }
    __syncthreads();
    bf16_t* Ct = (bf16_t*)p.Ct;
#pragma unroll 4
    for (int it = 0; it < (G2_BM * G2_BN / 8) / G2_THREADS; ++it) {
        const int idx = it * G2_THREADS + tid;
        const int r = idx >> 5, ch = idx & 31;
        if (row0 + r < row_end) {
            uint4 v = *(const uint4*)(smem + r * G2_EPI_ROW + ch * 16);
            *(uint4*)(Ct + (long)(row0 + r) * p.ldc + n0 + ch * 8) = v;
        }
    }
}

}  // namespace fpm
