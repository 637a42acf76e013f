// MFMA tile GEMM for gfx950, shared by every GEMM-shaped op of the matcher.
//
//   C[r, n] = epi( sum_seg  scale[r, seg] * sum_k A[row(r), k] * B_seg[n, k] )
//
// * A is M x K (K contiguous) with an optional row gather (edge -> source node for SplineConv).
// * B is N x K (K contiguous: weights pre-packed as [out][in]); with nseg > 1 the K loop walks
//   nseg segments, each with its own B matrix (SplineConv: the 4 B-spline cells of the edge's
//   group), and the segment partial sums are folded into the result with a per-row fp32 scale
//   (the B-spline basis) — so A rows are never rescaled or re-rounded.
// * Grouped mode (SplineConv): the row tile indexes a device-built tile table (group, first row);
//   entries past the real tile count have group -1 and exit.  With nseg == 1 the group selects
//   its B matrix (B + group * sB_seg): the (node, cell) product GEMM.
// * T = float  -> v_mfma_f32_16x16x4_f32  (exact fp32 products, parity mode)
//   T = bf16_t -> v_mfma_f32_16x16x32_bf16 (fp32 accumulate, throughput mode)
// Tile 128x128, 256 threads = 4 waves (2x2), 64x64 per wave = 4x4 MFMA 16x16 fragments.
// LDS double buffer with register-staged prefetch of the next K tile (one barrier per K tile).
#pragma once
#include "fpm_common.h"

namespace fpm {

enum GemmEpi : int {
    EPI_STORE = 0,      // v (+ bias)
    EPI_RELU = 1,       // relu(v + bias)
    EPI_TANH = 2,       // tanh(v + bias)
    EPI_AFFINITY = 3,   // C[j][i] = (j < n2b && i < n1b) ? softplus(v) - 0.5 : 0  (per pair)
    EPI_HALF_AFFINITY = 4,   // 0.5 * (softplus(v) - 0.5) on the same mask (quadratic Ke, ngm.py:289)
    EPI_NORM_MAX = 5,   // AFA-U block tail (gemm_big<128> only, fpm_gemm_norm_max): per 256-row
                        // tile = one pair, max_r InstanceNorm(res + v + bias) over the tile's rows
    EPI_NORM_OUT = 6,   // AFA-U block head (gemm_big<128> only, fpm_gemm_norm_out): InstanceNorm(v +
                        // bias) over each 256-row tile, to Cf (fp32) and Ct (bf16, ldt, zero K-pad)
};

struct GemmParams {
    const void* A;
    long lda, sA;            // row stride, batch stride (elements)
    const int* a_rows;       // optional row gather
    const void* B;
    long ldb, sB, sB_seg;    // row stride, batch stride, segment (cell) stride
    const float* row_scale;  // (rows, nseg) when nseg > 1
    int M, N, K, nseg;
    const int* tile_info;    // grouped: [tiles][2] = (group, row0)
    const int* group_off;    // grouped: group g rows are [group_off[g], group_off[g+1])
    int epi;
    const float* bias;
    float* Cf;
    void* Ct;
    long ldc, sC;
    const int* n1;
    const int* n2;
    int remap_mtiles;        // > 0: 1-D XCD-aware grid over remap_mtiles x ceil(N/128) tiles
    // EPI_NORM_MAX: residual rows (ldc stride), norm weight / bias, eps, per-pair max output (B x N)
    const float* res;
    const float* nw;
    const float* nb;
    float eps;
    float* gmax;
    long ldt;                // EPI_NORM_OUT / split: row stride of the bf16 copy Ct
    int split;               // > 0 (fp32-output 256-row kernels): Ct rows are split bf16 operands
    int norm_p;              // EPI_NORM_MAX / EPI_NORM_OUT: rows per pair, 256 (one tile) or 128 (two per tile); 0 = 256
                             // [hi | lo | hi] with segment stride split (ops.split_bf16x3 layout)
    int store_sc1;           // bf16 output tiles of the phase kernel: sc1 stores (the lines leave
                             // the XCD's L2 instead of evicting the gathered A rows)
    int remap_cm;            // phase kernel: row tiles per XCD chunk of the tile order (0 = 4)
};

// 1-D grid for the XCD-aware tile order: padded to whole rounds of 8 chunks so the remap is a
// bijection (extra blocks exit).
// Small launches (fewer than REMAP_MIN row tiles per batch) keep the plain order: dealing a
// handful of tiles in XCD chunks would put them all on one XCD.
constexpr int REMAP_MIN = 32;
inline unsigned remap_grid(int N, int mtiles) {
    long nt = (N + 127) / 128, chunk = 4 * nt;
    long t = nt * mtiles;
    if (mtiles < REMAP_MIN) return (unsigned)t;
    return (unsigned)((t + 8 * chunk - 1) / (8 * chunk) * (8 * chunk));
}
__device__ __forceinline__ int remap_tile(int nt, int mtiles, int cm = 4) {
    if (mtiles < REMAP_MIN) return blockIdx.x;
    const int chunk = cm * nt;
    const int i = blockIdx.x >> 3;
    return ((i / chunk) * 8 + (blockIdx.x & 7)) * chunk + (i % chunk);
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <typename T> struct TileCfg;
template <> struct TileCfg<float> {
    static constexpr int BK = 32;       // 128 B of K per row
    static constexpr int EPC = 4;       // elements per 16-B chunk
};
template <> struct TileCfg<bf16_t> {
    static constexpr int BK = 64;
    static constexpr int EPC = 8;
};

constexpr int GBM = 128, GBN = 128, GTHREADS = 256;
constexpr int LDS_ROW_BYTES = 144;      // 128 B of data + 16 B pad (bank spread)
constexpr int LDS_TILE_BYTES = GBM * LDS_ROW_BYTES;

// spline cell of B-spline corner s for group g = f0 + 5 f1 (open spline, kernel 5, degree 1)
__device__ __forceinline__ int spline_cell(int g, int s) {
    int f0 = g % 5, f1 = g / 5;
    return ((f0 + (s & 1)) % 5) + 5 * ((f1 + (s >> 1)) % 5);
}

template <typename T>
__device__ __forceinline__ void mfma_tile_step(const unsigned char* As, const unsigned char* Bs, int wm, int wn,
                                               int lane, f32x4_t (&acc)[4][4]);

template <>
__device__ __forceinline__ void mfma_tile_step<bf16_t>(const unsigned char* As, const unsigned char* Bs, int wm,
                                                       int wn, int lane, f32x4_t (&acc)[4][4]) {
    const int r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        bf16x8_t a[4], b[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            a[f] = *(const bf16x8_t*)(As + (wm * 64 + f * 16 + r) * LDS_ROW_BYTES + (kk * 32 + q * 8) * 2);
            b[f] = *(const bf16x8_t*)(Bs + (wn * 64 + f * 16 + r) * LDS_ROW_BYTES + (kk * 32 + q * 8) * 2);
        }
#pragma unroll
        for (int fm = 0; fm < 4; ++fm)
#pragma unroll
            for (int fn = 0; fn < 4; ++fn)
                acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[fm], b[fn], acc[fm][fn], 0, 0, 0);
    }
}

template <>
__device__ __forceinline__ void mfma_tile_step<float>(const unsigned char* As, const unsigned char* Bs, int wm,
                                                      int wn, int lane, f32x4_t (&acc)[4][4]) {
    const int r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
        f32x4_t a[4], b[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            a[f] = *(const f32x4_t*)(As + (wm * 64 + f * 16 + r) * LDS_ROW_BYTES + (kc * 16 + q * 4) * 4);
            b[f] = *(const f32x4_t*)(Bs + (wn * 64 + f * 16 + r) * LDS_ROW_BYTES + (kc * 16 + q * 4) * 4);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < 4; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[fm][t], b[fn][t], acc[fm][fn], 0, 0, 0);
    }
}

template <typename T, bool SEGSCALE>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_kernel(GemmParams p) {
    constexpr int BK = TileCfg<T>::BK;
    constexpr int EPC = TileCfg<T>::EPC;
    __shared__ __attribute__((aligned(16))) unsigned char smem[4 * LDS_TILE_BYTES];
#define AS_(buf) (smem + (buf) * LDS_TILE_BYTES)
#define BS_(buf) (smem + (2 + (buf)) * LDS_TILE_BYTES)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int batch = blockIdx.z;
    int ntile = blockIdx.x, mtile = blockIdx.y;
    if (p.remap_mtiles > 0) {
        // Workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8).  Give each XCD a
        // contiguous run of logical tiles, N fastest, so the ceil(N/128) column tiles that share an
        // A row-tile (and consecutive row tiles sharing a weight) hit the same XCD's L2.
        // Runs are chunks of 4 row tiles x nt column tiles, dealt to the XCDs in turn, so a tail of
        // empty tiles (grouped mode over-provisions the table) stays spread over all 8 XCDs.
        const int nt = (p.N + GBN - 1) / GBN;
        const int q = remap_tile(nt, p.remap_mtiles);
        mtile = q / nt;
        ntile = q - mtile * nt;
        if (mtile >= p.remap_mtiles) return;
    }
    const int n0 = ntile * GBN;

    int group = 0, row0, row_end;
    if (p.tile_info) {
        group = p.tile_info[2 * mtile];
        if (group < 0) return;
        row0 = p.tile_info[2 * mtile + 1];
        row_end = p.group_off[group + 1];
    } else {
        row0 = mtile * GBM;
        row_end = p.M;
    }

    const T* A = (const T*)p.A + (long)batch * p.sA;
    const T* Bb = (const T*)p.B + (long)batch * p.sB;

    // per-thread load slots: chunk c (16 B) of rows (tid>>3) + 32*i
    const int lc = tid & 7;
    long a_off[4];
    int b_row[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int r = row0 + (tid >> 3) + 32 * i;
        int rr = r < row_end ? r : row0;            // clamp (rows past the end are never stored)
        long arow = p.a_rows ? (long)p.a_rows[rr] : (long)rr;
        a_off[i] = arow * p.lda;
        int n = n0 + (tid >> 3) + 32 * i;
        b_row[i] = n < p.N ? n : 0;
    }
    const int ktiles = (p.K + BK - 1) / BK;
    const int total = ktiles * p.nseg;

    uint4 ra[4], rb[4];
    auto load_tile = [&](int kt) {
        int seg = kt / ktiles;
        int k0 = (kt - seg * ktiles) * BK + lc * EPC;
        const T* Bseg = Bb + (long)(p.nseg > 1 ? spline_cell(group, seg) : group) * p.sB_seg;
        bool kin = k0 < p.K;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            ra[i] = kin ? *(const uint4*)(A + a_off[i] + k0) : make_uint4(0, 0, 0, 0);
            rb[i] = kin ? *(const uint4*)(Bseg + (long)b_row[i] * p.ldb + k0) : make_uint4(0, 0, 0, 0);
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int r = (tid >> 3) + 32 * i;
            *(uint4*)(AS_(buf) + r * LDS_ROW_BYTES + lc * 16) = ra[i];
            *(uint4*)(BS_(buf) + r * LDS_ROW_BYTES + lc * 16) = rb[i];
        }
    };

    f32x4_t acc[4][4];
    f32x4_t res[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            res[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }

    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < total; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < total) load_tile(kt + 1);
        mfma_tile_step<T>(AS_(cur), BS_(cur), wm, wn, lane, acc);
        if (SEGSCALE) {
            int seg = kt / ktiles;
            if (kt - seg * ktiles == ktiles - 1) {   // segment complete: res += basis[r, seg] * acc
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        int r = row0 + wm * 64 + fm * 16 + (lane >> 4) * 4 + j;
                        float sc = r < row_end ? p.row_scale[(long)r * p.nseg + seg] : 0.f;
#pragma unroll
                        for (int fn = 0; fn < 4; ++fn) {
                            res[fm][fn][j] += sc * acc[fm][fn][j];
                            acc[fm][fn][j] = 0.f;
                        }
                    }
                }
            }
        }
        if (kt + 1 < total) store_tile(cur ^ 1);
        __syncthreads();
    }

#undef AS_
#undef BS_
    // epilogue
    constexpr bool BF16OP = sizeof(T) == 2;
    const int epi = p.epi;
    int n1b = 0, n2b = 0;
    if (epi == EPI_AFFINITY || epi == EPI_HALF_AFFINITY) { n1b = p.n1[batch]; n2b = p.n2[batch]; }
    float* Cf = p.Cf ? p.Cf + (long)batch * p.sC : nullptr;
    T* Ct = p.Ct ? (T*)p.Ct + (long)batch * p.sC : nullptr;
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = row0 + wm * 64 + fm * 16 + (lane >> 4) * 4 + j;
            if (r >= row_end) continue;
#pragma unroll
            for (int fn = 0; fn < 4; ++fn) {
                const int n = n0 + wn * 64 + fn * 16 + (lane & 15);
                if (n >= p.N) continue;
                float v = SEGSCALE ? res[fm][fn][j] : acc[fm][fn][j];
                if (p.bias) v += p.bias[n];
                if (epi == EPI_RELU) v = fmaxf(v, 0.f);
                else if (epi == EPI_TANH) v = tanhf(v);
                // bf16 operands: the same softplus as the 256-row kernels' affinity epilogue
                // (gemm_big.h), so a pair's Kp does not depend on which kernel its batch size picks
                else if (epi == EPI_AFFINITY)
                    v = (r < n2b && n < n1b) ? (BF16OP ? softplus_fast(v) : softplus_f(v)) - 0.5f : 0.f;
                else if (epi == EPI_HALF_AFFINITY)
                    v = (r < n2b && n < n1b) ? 0.5f * ((BF16OP ? softplus_fast(v) : softplus_f(v)) - 0.5f) : 0.f;
                long o = (long)r * p.ldc + n;
                if (Cf) Cf[o] = v;
                if (Ct) Ct[o] = from_f<T>(v);
            }
        }
    }
}

}  // namespace fpm
