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
//   * per K step of BK, the weight tile (256 rows) and both token tiles (hi, lo: 128 rows each)
//     go L2 -> LDS by global_load_lds_dwordx4 (1 KiB per wave-instruction) into a ring of NS
//     stages, NS - 1 steps ahead of the multiply: the wait for step kt is a counted
//     `s_waitcnt vmcnt` that leaves the later steps' DMA in flight, then a raw s_barrier (a
//     __syncthreads() would drain every DMA), and the refill goes into the stage every wave
//     finished reading before that barrier;
//   * LDS image: rows of BK f16, 16-B chunk c of row r at chunk position c ^ f(r) (f = (r >> 1) & 7
//     for 8-chunk rows, (r >> 2) & 3 for 4-chunk rows), so each ds_read_b128 lane group (16
//     distinct rows, one chunk) hits 16 distinct 16-B bank slots (the DMA writes lane-linearly,
//     so the permutation is applied to the per-lane SOURCE address and undone on the read);
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
constexpr int MM_THREADS = 512;  // 8 waves
constexpr int MM_BK = 64;        // k per stage of the default instantiation (mm_f16_kernel below)
constexpr int MM_NS = 2;         // stages of the default instantiation
constexpr int MM_FL = 12;        // flags of the default instantiation: 16x16x32 tiles, grouped tile order
constexpr int MM_KMULT = 64;     // K (and every K slice) in whole multiples of this
__host__ __device__ constexpr int mm_stage_bytes(const int bk) { return (MM_BR + 2 * MM_BT) * bk * 2; }
constexpr int MM_LDS = MM_NS * mm_stage_bytes(MM_BK);

typedef _Float16 mm_f16x8 __attribute__((ext_vector_type(8)));
typedef float mm_f32x16 __attribute__((ext_vector_type(16)));
typedef float mm_f32x4 __attribute__((ext_vector_type(4)));

struct MmArgs {
    const uint16_t* w;   // [rows][K] f16 bits
    const uint16_t* xh;  // [n][K]
    const uint16_t* xl;  // [n][K]
    float* out;          // [ks][n][rows]
    int rows, K, n, ks;  // K % (ks * BK) == 0 (host-checked)
    int n_rt, n_tt;      // tiles: ceil(rows / MM_BR), ceil(n / MM_BT)
};

__host__ __device__ constexpr int mm_row_tiles(const int rows) { return (rows + MM_BR - 1) / MM_BR; }
__host__ __device__ constexpr int mm_tok_tiles(const int n, const int bt = MM_BT) { return (n + bt - 1) / bt; }
// K slices (1, 2, 4, 8): minimise the modelled time rounds(ks) * (1 / ks + MM_WG_FIXED), rounds =
// ceil(tiles * ks / n_cu) (workgroups over the CUs) and MM_WG_FIXED a workgroup's fixed cost
// (prologue, partial stores, tail) in units of one full-K tile, fitted to tools/gemm_bench on
// MI355X (e.g. qkv at 2048 tokens: 384 tiles are 1.5 rounds, split 2-way 3 even rounds, -7 %;
// W1/W3 at 512 tokens split 4-way +14 %); K in whole 64-deep steps per slice and
// ks * n * rows <= max_floats (the partials buffer); 0 if K is not a multiple of 64
constexpr double MM_WG_FIXED = 0.15;
inline int mm_pick_ks(const int rows, const int K, const int n, const size_t max_floats, const int n_cu = 256,
                      const int bt = MM_BT) {
    if (K % MM_KMULT) return 0;
    const int tiles = mm_row_tiles(rows) * mm_tok_tiles(n, bt);
    int best = 1;
    double best_t = 1e30;
    for (int ks = 1; ks <= 8; ks *= 2) {
        if (K % (ks * MM_KMULT) || (size_t)ks * n * rows > max_floats) break;
        const double t = (double)((tiles * ks + n_cu - 1) / n_cu) * (1.0 / ks + MM_WG_FIXED);
        if (t < best_t * 0.999) {
            best_t = t;
            best = ks;
        }
    }
    return best;
}

typedef __attribute__((address_space(3))) void* mm_lds_ptr;

template <int N>
__device__ __forceinline__ void mm_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BK, int NS, int BT = 128, int NW = 8>
struct MmCfg {
    static constexpr int RB = BK * 2;             // LDS image row bytes
    static constexpr int CH = RB / 16;            // 16-B chunks per row
    static constexpr int RPI = 1024 / RB;         // image rows per DMA wave-instruction
    static constexpr int SH = CH == 8 ? 1 : 2;    // swizzle f(r) = (r >> SH) & (CH - 1)
    static constexpr int STAGE = (MM_BR + 2 * BT) * RB;
    static constexpr int WI = MM_BR / RPI / NW;   // W instructions per wave per stage
    static constexpr int XI = BT / RPI / NW;      // Xh (and Xl) instructions per wave per stage
    static constexpr int LPS = WI + 2 * XI;       // DMA instructions per wave per stage
    static constexpr int LDS = NS * STAGE;
    static constexpr int WT = BT / 64;            // waves along the tokens (64 tokens each)
    static constexpr int WR = NW / WT;            // waves along the rows
    static constexpr int RT = MM_BR / WR / 32;    // 32-row tiles per wave
    static_assert(BK == 32 || BK == 64, "BK");
    static_assert(BT == 128 || BT == 256, "BT");
    static_assert((NW == 8 || NW == 4) && XI >= 1 && WR >= 1, "NW");
    static_assert(NS >= 2 && LDS <= 160 * 1024, "stages");
    __device__ static uint32_t off(const int r, const int c) { return (uint32_t)(r * RB + 16 * (c ^ ((r >> SH) & (CH - 1)))); }
};

// the wait before step kt: `ahead` later steps' DMA may stay in flight (ahead = 0 .. NS - 2)
template <int LPS, int NS>
__device__ __forceinline__ void mm_wait_ahead(const int ahead) {
    if constexpr (NS >= 5) { if (ahead >= 3) { mm_wait_vm<3 * LPS>(); return; } }
    if constexpr (NS >= 4) { if (ahead >= 2) { mm_wait_vm<2 * LPS>(); return; } }
    if constexpr (NS >= 3) { if (ahead >= 1) { mm_wait_vm<LPS>(); return; } }
    mm_wait_vm<0>();
}

// FL bit 0: a k-step's next fragments read before its current MFMAs; bit 1: s_setprio(1) around
// the MFMA clusters; bit 3: 16x16x32 MFMA tiles (BK 64); bit 2: grouped tile order (8 row tiles x n_tt token tiles per group, row tile
// fastest: the 32 workgroups an XCD runs at once cover 8 x 4 tiles, sharing both operands in L2)
// OCC: waves per SIMD the register allocation must allow (2: one 512-thread workgroup per CU;
// 4: two, each with at most 80 KiB of LDS).  NW: waves per workgroup, 8 (2 x 4 waves of 64 x 64)
// or 4 (2 x 2 waves of 64 tokens x 128 rows: a third less LDS read per MFMA)
template <int BK, int NS, int FL, int BT = 128, int OCC = 2, int NW = 8>
__global__ __launch_bounds__(64 * NW, OCC) void mm_f16_kernel_t(const MmArgs a) {
    using C = MmCfg<BK, NS, BT, NW>;
    extern __shared__ __attribute__((aligned(16))) char mm_smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    // bijective XCD-major order: blocks b and b + 8 share an XCD; consecutive L share one
    const int nb = gridDim.x, b = blockIdx.x;
    const int q = nb >> 3, rem = nb & 7, xcd = b & 7;
    const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
    int tt, R;  // token tile, row tile x slice (R = rt * ks + s)
    if constexpr (FL & 4) {
        constexpr int GR = 8;
        const int n_R = a.n_rt * a.ks, per_group = GR * a.n_tt;
        const int grp = L / per_group, in = L - grp * per_group;
        const int gr = min(n_R - grp * GR, GR);
        R = grp * GR + in % gr;
        tt = in / gr;
    } else {
        tt = L % a.n_tt;
        R = L / a.n_tt;
    }
    const int s = R % a.ks, rt = R / a.ks;
    const int row0 = rt * MM_BR, t0 = tt * BT;
    const int kslice = a.K / a.ks, kbeg = s * kslice, nk = kslice / BK;
    const size_t K = (size_t)a.K;

    // this lane's DMA sources (rows / tokens past the end clamped: valid memory whose products
    // are never stored) and chunk: image row r0 + lane / CH, chunk position lane % CH holding
    // source chunk (lane % CH) ^ f(row)
    const uint16_t* wsrc[C::WI];
    const uint16_t* hsrc[C::XI];
    const uint16_t* lsrc[C::XI];
#pragma unroll
    for (int i = 0; i < C::WI; i++) {
        const int r = (wv * C::WI + i) * C::RPI + lane / C::CH;
        const int c = (lane % C::CH) ^ ((r >> C::SH) & (C::CH - 1));
        wsrc[i] = a.w + (size_t)min(row0 + r, a.rows - 1) * K + kbeg + 8 * c;
    }
#pragma unroll
    for (int i = 0; i < C::XI; i++) {
        const int r = (wv * C::XI + i) * C::RPI + lane / C::CH;
        const int c = (lane % C::CH) ^ ((r >> C::SH) & (C::CH - 1));
        const size_t o = (size_t)min(t0 + r, a.n - 1) * K + kbeg + 8 * c;
        hsrc[i] = a.xh + o;
        lsrc[i] = a.xl + o;
    }
    auto issue = [&](const int stage, const int kt) {
        char* base = mm_smem + stage * C::STAGE;
        const int k = kt * BK;
#pragma unroll
        for (int i = 0; i < C::WI; i++)
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k), (mm_lds_ptr)(base + (wv * C::WI + i) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int i = 0; i < C::XI; i++)
            __builtin_amdgcn_global_load_lds((const void*)(hsrc[i] + k),
                                             (mm_lds_ptr)(base + MM_BR * C::RB + (wv * C::XI + i) * 1024), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < C::XI; i++)
            __builtin_amdgcn_global_load_lds((const void*)(lsrc[i] + k),
                                             (mm_lds_ptr)(base + (MM_BR + BT) * C::RB + (wv * C::XI + i) * 1024), 16,
                                             0, 0);
    };

    constexpr int RT = C::RT;
    const int wt = wv / C::WR, wr = wv % C::WR;  // this wave's 64 tokens / RT x 32 rows of the tile
    if constexpr (FL & 8) {
        // v_mfma_f32_16x16x32_f16 (the microarch guide: ~1.15x the FLOP/s of 32x32x16 at equal
        // cycles per FLOP, the chip holds a higher clock): 4 x 2RT tiles of 16 x 16 per wave; lane l
        // reads row l & 15 at chunk 4 q + (l >> 4) of a 32-deep step q (the same image stays
        // conflict-free: a lane group covers rows 0-3, 12-15 at one chunk and 4-11 at the next)
        static_assert(BK % 32 == 0, "16x16x32 tiles read 32-deep steps");
        constexpr int RS = 2 * RT;  // 16-row tiles per wave
        const int l16 = lane & 15, q4 = lane >> 4;
        mm_f32x4 acc4[4][RS];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < RS; j++) acc4[i][j] = mm_f32x4{};
        struct F16 { mm_f16x8 ah[4], al[4], bw[RS]; };
        auto load16 = [&](const char* base, const int q, F16& f) {
            const char* w_img = base;
            const char* xh_img = base + MM_BR * C::RB;
            const char* xl_img = base + (MM_BR + BT) * C::RB;
            const int c = 4 * q + q4;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t o = C::off(64 * wt + 16 * i + l16, c);
                f.ah[i] = *(const mm_f16x8*)(xh_img + o);
                f.al[i] = *(const mm_f16x8*)(xl_img + o);
            }
#pragma unroll
            for (int j = 0; j < RS; j++) f.bw[j] = *(const mm_f16x8*)(w_img + C::off(32 * RT * wr + 16 * j + l16, c));
        };
        auto mma16 = [&](const F16& f) {
            if constexpr (FL & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < RS; j++) {
                    acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.ah[i], f.bw[j], acc4[i][j], 0, 0, 0);
                    acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.al[i], f.bw[j], acc4[i][j], 0, 0, 0);
                }
            if constexpr (FL & 2) __builtin_amdgcn_s_setprio(0);
        };
        auto compute16 = [&](const int stage) {
            const char* base = mm_smem + stage * C::STAGE;
            if constexpr (FL & 1) {
                // the next 32-deep step's fragments requested before this one's MFMAs
                F16 f0, f1;
                load16(base, 0, f0);
#pragma unroll
                for (int q = 0; q < BK / 32; q++) {
                    if (q + 1 < BK / 32) load16(base, q + 1, (q & 1) ? f0 : f1);
                    mma16((q & 1) ? f1 : f0);
                }
                return;
            }
            const char* w_img = base;
            const char* xh_img = base + MM_BR * C::RB;
            const char* xl_img = base + (MM_BR + BT) * C::RB;
#pragma unroll
            for (int q = 0; q < BK / 32; q++) {
                const int c = 4 * q + q4;
                mm_f16x8 ah[4], al[4], bw[RS];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t o = C::off(64 * wt + 16 * i + l16, c);
                    ah[i] = *(const mm_f16x8*)(xh_img + o);
                    al[i] = *(const mm_f16x8*)(xl_img + o);
                }
#pragma unroll
                for (int j = 0; j < RS; j++) bw[j] = *(const mm_f16x8*)(w_img + C::off(32 * RT * wr + 16 * j + l16, c));
                if constexpr (FL & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < RS; j++) {
                        acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bw[j], acc4[i][j], 0, 0, 0);
                        acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bw[j], acc4[i][j], 0, 0, 0);
                    }
                if constexpr (FL & 2) __builtin_amdgcn_s_setprio(0);
            }
        };
#pragma unroll
        for (int d = 0; d < NS - 1; d++)
            if (d < nk) issue(d, d);
        for (int kt = 0; kt < nk; kt++) {
            mm_wait_ahead<C::LPS, NS>(min(NS - 2, nk - 1 - kt));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own ds_reads of the refilled stage retired
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (kt + NS - 1 < nk) issue((kt + NS - 1) % NS, kt + NS - 1);
            compute16(kt % NS);
        }
        // D: lane l holds row l & 15 of a 16 x 16 tile for tokens 4 (l >> 4) + reg
        float* out = a.out + (size_t)s * a.n * a.rows;
#pragma unroll
        for (int j = 0; j < RS; j++) {
            const int r = row0 + 32 * RT * wr + 16 * j + l16;
            if (r >= a.rows) continue;
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int reg = 0; reg < 4; reg++) {
                    const int t = t0 + 64 * wt + 16 * i + 4 * q4 + reg;
                    if (t < a.n) out[(size_t)t * a.rows + r] = acc4[i][j][reg];
                }
        }
        return;
    }
    mm_f32x16 acc[2][RT];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < RT; j++) acc[i][j] = mm_f32x16{};
    struct Frags { mm_f16x8 ah[2], al[2], bw[RT]; };
    auto load_frags = [&](const char* base, const int kk, Frags& f) {
        const char* w_img = base;
        const char* xh_img = base + MM_BR * C::RB;
        const char* xl_img = base + (MM_BR + BT) * C::RB;
        const int c = 2 * kk + h;
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const uint32_t o = C::off(64 * wt + 32 * i + l32, c);
            f.ah[i] = *(const mm_f16x8*)(xh_img + o);
            f.al[i] = *(const mm_f16x8*)(xl_img + o);
        }
#pragma unroll
        for (int j = 0; j < RT; j++) f.bw[j] = *(const mm_f16x8*)(w_img + C::off(32 * RT * wr + 32 * j + l32, c));
    };
    auto mma = [&](const Frags& f) {
        if constexpr (FL & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < RT; j++) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[i], f.bw[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.al[i], f.bw[j], acc[i][j], 0, 0, 0);
            }
        if constexpr (FL & 2) __builtin_amdgcn_s_setprio(0);
    };
    auto compute = [&](const int stage) {
        const char* base = mm_smem + stage * C::STAGE;
        if constexpr (FL & 1) {
            // the next 16-deep step's fragments requested before this one's MFMAs
            Frags f0, f1;
            load_frags(base, 0, f0);
#pragma unroll
            for (int kk = 0; kk < BK / 16; kk++) {
                if (kk + 1 < BK / 16) load_frags(base, kk + 1, (kk & 1) ? f0 : f1);
                mma((kk & 1) ? f1 : f0);
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < BK / 16; kk++) {
                Frags f;
                load_frags(base, kk, f);
                mma(f);
            }
        }
    };

    // ring of NS stages, NS - 1 steps of DMA ahead of the multiply
#pragma unroll
    for (int d = 0; d < NS - 1; d++)
        if (d < nk) issue(d, d);
    for (int kt = 0; kt < nk; kt++) {
        mm_wait_ahead<C::LPS, NS>(min(NS - 2, nk - 1 - kt));  // this wave's DMA of step kt landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own ds_reads of the refilled stage retired
        __builtin_amdgcn_s_barrier();                          // ... every wave's; stage kt - 1 read
        asm volatile("" ::: "memory");
        if (kt + NS - 1 < nk) issue((kt + NS - 1) % NS, kt + NS - 1);
        compute(kt % NS);
    }

    // D: lane l holds row l & 31, tokens (reg & 3) + 8 (reg >> 2) + 4 h of each 32 x 32 tile
    float* out = a.out + (size_t)s * a.n * a.rows;
#pragma unroll
    for (int j = 0; j < RT; j++) {
        const int r = row0 + 32 * RT * wr + 32 * j + l32;
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

// the product's instantiations: the default, and for launches of >= MM_W4_PER_CU workgroups per
// CU (W1/W3 and the lm_head at 2048 tokens) two 4-wave workgroups per CU with 32-deep steps in
// 64 KiB each, every wave 64 tokens x 128 rows (tools/gemm_bench, 2048 tokens: W1/W3 840 -> 809
// us; qkv, Wo, W2 slower, their launches have 1-3 workgroups per CU).  Inside a K slice both
// sum each accumulator in the same k order (32-deep MFMA steps, hi then lo); the K-slice count
// is picked per instantiation (mm_pick_ks with its token tile), so the two can differ in the
// last bits of a partial sum.  Which one runs depends on the launch's workgroups per CU (the
// device's CU count): tests compare either against the float64 product, not against each other.
#define mm_f16_kernel mm_f16_kernel_t<MM_BK, MM_NS, MM_FL, MM_BT>
#define mm_f16_kernel_w4 mm_f16_kernel_t<32, 2, MM_FL, MM_BT, 2, 4>
constexpr int MM_LDS_W4 = MmCfg<32, 2, MM_BT, 4>::LDS;
constexpr int MM_THREADS_W4 = 256;
constexpr int MM_W4_PER_CU = 4;

}  // namespace xalm
