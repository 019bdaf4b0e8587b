// gemm16.h — the prompt-pass GEMM (the prompt loop it replaces is
// jubruckne/Xalm src/main.cpp:94-100, each token a matmul of src/infer.cpp:104-135).
//
//   Y[t][r] = sum_k W[r][k] * (Xh[t][k] + Xl[t][k])        (Xh + Xl: one activation row, split)
//
// W is a weight matrix as uploaded ([rows][K] f16; fp8 matrices reach it as their exact f16 image),
// Xh / Xl the exact f16 hi / lo halves of the pass's activation rows under a power-of-two row scale
// (prefill.h: |x - (hi + lo) / s| <= 2^-22 |x|).  f16 x f16 products are exact in the f32
// accumulator of v_mfma_f32_32x32x16_f16, hi and lo accumulate into the SAME accumulator, and the
// epilogue kernel multiplies by 1 / s_t.  Summation order is fixed by the tiling (no atomics, no
// run-time algorithm choice): the same inputs give the same bits on every run.
//
// Tiling (MI355X: 256 CUs, 160 KiB LDS, 64-wide waves):
//   * a workgroup owns 256 weight rows x 128 tokens and one K slice (split-K partials
//     [slice][t][r], summed in slice order by the epilogue); 512 threads = 8 waves as 2 (tokens)
//     x 4 (rows), each wave 64 tokens x 64 rows = 2 x 2 tiles of 32 x 32 (64 f32 accumulators);
//   * per K step of 64, the weight tile (256 x 128 B = 32 KiB) and both token tiles (2 x 16 KiB)
//     go HBM/L2 -> LDS by global_load_lds_dwordx4 (1 KiB per wave-instruction, 8 per wave), into
//     the second of two 64 KiB LDS stages while the waves multiply the first;
//   * LDS image: 128-B rows, 16-B chunk c of row r at chunk position c ^ ((r >> 1) & 7), so each
//     ds_read_b128 lane group (16 distinct rows, one chunk) hits 16 distinct 16-B bank slots (the
//     DMA writes lane-linearly, so the permutation is applied to the per-lane SOURCE address and
//     undone on the read);
//   * MFMA operands: A = tokens (lane: token l & 31, k = 8 (l >> 5) + j), B = weight rows (lane:
//     row l & 31, same k); D lane l holds row l & 31 for tokens (reg & 3) + 8 (reg >> 2) + 4 (l >> 5),
//     so a store instruction writes 32 consecutive rows (128 B) of two tokens;
//   * workgroup -> tile: the token tiles of one (row tile, slice) are consecutive in a
//     bijective XCD-major order, so they share an XCD (its L2 serves the weight tile's re-reads).
#pragma once

#include "common.h"

namespace xalm {

constexpr int MM_BR = 256;       // weight rows per workgroup
constexpr int MM_BT = 128;       // tokens per workgroup
constexpr int MM_BK = 64;        // k per stage: 128-byte LDS rows
constexpr int MM_THREADS = 512;  // 8 waves
constexpr int MM_STAGE = (MM_BR + 2 * MM_BT) * MM_BK * 2;  // bytes: W, Xh, Xl tiles
constexpr int MM_LDS = 2 * MM_STAGE;                       // 128 KiB

typedef _Float16 mm_f16x8 __attribute__((ext_vector_type(8)));
typedef float mm_f32x16 __attribute__((ext_vector_type(16)));

struct MmArgs {
    const uint16_t* w;   // [rows][K] f16 bits
    const uint16_t* xh;  // [n][K]
    const uint16_t* xl;  // [n][K]
    float* out;          // [ks][n][rows]
    int rows, K, n, ks;  // K % (ks * MM_BK) == 0 (host-checked)
    int n_rt, n_tt;      // tiles: ceil(rows / MM_BR), ceil(n / MM_BT)
};

__host__ __device__ constexpr int mm_row_tiles(const int rows) { return (rows + MM_BR - 1) / MM_BR; }
__host__ __device__ constexpr int mm_tok_tiles(const int n) { return (n + MM_BT - 1) / MM_BT; }
// K slices: doubled (up to 8) while the grid is under 3/4 of the 256 CUs, K splits into whole
// 64-deep steps and the partials fit (ks * n <= max_ks_n); 0 if K is not a multiple of MM_BK
inline int mm_pick_ks(const int rows, const int K, const int n, const int max_ks_n) {
    if (K % MM_BK) return 0;
    const int tiles = mm_row_tiles(rows) * mm_tok_tiles(n);
    int ks = 1;
    while (ks < 8 && tiles * ks < 192 && K % (2 * ks * MM_BK) == 0 && 2 * ks * n <= max_ks_n) ks *= 2;
    return ks;
}

// byte offset of 16-B chunk c (0..7) of LDS image row r
__device__ __forceinline__ uint32_t mm_lds_off(const int r, const int c) {
    return (uint32_t)(r * 128 + 16 * (c ^ ((r >> 1) & 7)));
}

typedef __attribute__((address_space(3))) void* mm_lds_ptr;

// One wave-instruction: image rows r0 .. r0 + 7 of a tile from `src` rows (row pitch K elements),
// lane l -> image row r0 + (l >> 3), chunk position l & 7 (holding source chunk (l & 7) ^ swz).
__device__ __forceinline__ void mm_issue8(const uint16_t* src_rows, const size_t K, const int r0, const int lane,
                                          char* lds_tile, const int src_row, const int k) {
    const int r = r0 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const uint16_t* g = src_rows + (size_t)src_row * K + k + 8 * c;
    __builtin_amdgcn_global_load_lds((const void*)g, (mm_lds_ptr)(lds_tile + r0 * 128), 16, 0, 0);
}

__global__ __launch_bounds__(MM_THREADS, 2) void mm_f16_kernel(const MmArgs a) {
    extern __shared__ __attribute__((aligned(16))) char mm_smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    // bijective XCD-major order: blocks b and b + 8 share an XCD; consecutive L share one
    const int nb = gridDim.x, b = blockIdx.x;
    const int q = nb >> 3, rem = nb & 7, xcd = b & 7;
    const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
    const int tt = L % a.n_tt, rest = L / a.n_tt;
    const int s = rest % a.ks, rt = rest / a.ks;
    const int row0 = rt * MM_BR, t0 = tt * MM_BT;
    const int kslice = a.K / a.ks, kbeg = s * kslice, nk = kslice / MM_BK;
    const size_t K = (size_t)a.K;

    // this lane's source rows for its 8 DMA instructions per stage (clamped: rows / tokens past
    // the end load valid memory whose products are never stored)
    int wsrc[4], xsrc[2];
#pragma unroll
    for (int i = 0; i < 4; i++) wsrc[i] = min(row0 + 32 * wv + 8 * i + (lane >> 3), a.rows - 1);
#pragma unroll
    for (int i = 0; i < 2; i++) xsrc[i] = min(t0 + 16 * wv + 8 * i + (lane >> 3), a.n - 1);
    auto issue = [&](const int stage, const int k) {
        char* base = mm_smem + stage * MM_STAGE;
#pragma unroll
        for (int i = 0; i < 4; i++) mm_issue8(a.w, K, 32 * wv + 8 * i, lane, base, wsrc[i], k);
#pragma unroll
        for (int i = 0; i < 2; i++) mm_issue8(a.xh, K, 16 * wv + 8 * i, lane, base + MM_BR * 128, xsrc[i], k);
#pragma unroll
        for (int i = 0; i < 2; i++) mm_issue8(a.xl, K, 16 * wv + 8 * i, lane, base + (MM_BR + MM_BT) * 128, xsrc[i], k);
    };

    const int wt = wv >> 2, wr = wv & 3;  // this wave's 64 tokens / 64 rows of the tile
    mm_f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = mm_f32x16{};
    auto compute = [&](const int stage) {
        const char* base = mm_smem + stage * MM_STAGE;
        const char* wt_img = base;
        const char* xh_img = base + MM_BR * 128;
        const char* xl_img = base + (MM_BR + MM_BT) * 128;
#pragma unroll
        for (int kk = 0; kk < MM_BK / 16; kk++) {
            const int c = 2 * kk + h;
            mm_f16x8 ah[2], al[2], bw[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const uint32_t o = mm_lds_off(64 * wt + 32 * i + l32, c);
                ah[i] = *(const mm_f16x8*)(xh_img + o);
                al[i] = *(const mm_f16x8*)(xl_img + o);
            }
#pragma unroll
            for (int j = 0; j < 2; j++) bw[j] = *(const mm_f16x8*)(wt_img + mm_lds_off(64 * wr + 32 * j + l32, c));
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bw[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bw[j], acc[i][j], 0, 0, 0);
                }
        }
    };

    // two stages: the DMA of step kt + 1 runs under the MFMAs of step kt
    issue(0, kbeg);
    for (int kt = 0; kt < nk; kt++) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // stage kt & 1 landed for every wave; stage (kt + 1) & 1 no longer read
        if (kt + 1 < nk) issue((kt + 1) & 1, kbeg + (kt + 1) * MM_BK);
        compute(kt & 1);
    }

    // D: lane l holds row l & 31, tokens (reg & 3) + 8 (reg >> 2) + 4 h of each 32 x 32 tile
    float* out = a.out + (size_t)s * a.n * a.rows;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int r = row0 + 64 * wr + 32 * j + l32;
        if (r >= a.rows) continue;
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int reg = 0; reg < 16; reg++) {
                const int t = t0 + 64 * wt + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                if (t < a.n) out[(size_t)t * a.rows + r] = acc[i][j][reg];
            }
    }
}

}  // namespace xalm
