// prefill.h — batched prompt processing: the prompt loop of run_completion
// (jubruckne/Xalm src/main.cpp:94-100, HYDRATE_KV_CACHE src/infer.cpp:620-623) for up to
// PF_TOK tokens per pass, so every weight matrix is streamed once per pass instead of once
// per token.  Same math per token as the decode path (src/infer.cpp:365-496); the matrix
// products run on the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 products, f32
// accumulation — a k-ordered fmaf chain, MI355X_MICROARCH.md "Matrix cores"), so activations
// stay f32 exactly as in the reference and only the summation order differs — or, for fp8
// weights by default (XH_OPT_PREFILL), on the split-f16 MFMA below (activations as exact
// f16 hi + lo pairs, ≈22-bit mantissa).
//
// GEMM layout: Y[t][r] = sum_k X[t][k] W[r][k], W row-major [rows][K] as uploaded.  One wave
// owns RT 32-row tiles x one K slice x up to 64 tokens (2 RT 32x32 f32 accumulators).  Lane l
// streams 16 bytes of row r0 + (l & 31) at k = kb + E (l >> 5) and decodes them to E floats:
// they are the B operand of E MFMAs whose A operand is X[t][same k] (MFMA 32x32x2 f32 operand
// map: A[i = l & 31][k = l >> 5], B[k = l >> 5][j = l & 31]), so weights go HBM -> VGPR ->
// MFMA with no LDS staging; X (a few MB) is read from L2 (a transposed X^T layout, whose
// A-operand loads read whole 128-B lines, measured no faster: +1 % f16, -7 % fp8).  K slices
// write f32 partials
// [slice][t][r]; a second kernel sums them in slice order and applies the decode path's
// epilogue (clip + rope + fp16 K/V write, silu * up, residual add).
#pragma once

#include "attention.h"
#include "gemm16.h"
#include "gemv.h"

namespace xalm {

constexpr int PF_TOK = 64;       // tokens per pass of the hand-written MFMA GEMMs (two token tiles)
constexpr int PF_TOK_MM = 2048;  // tokens per pass of the LDS-tiled f16 GEMM (gemm16.h)
constexpr int PF_TOK_BLAS = 512; // tokens per pass of the hipBLASLt GEMMs (XH_OPT_PREFILL 4)
constexpr int PF_TOK_MAX = PF_TOK_MM > PF_TOK_BLAS ? PF_TOK_MM : PF_TOK_BLAS;
constexpr int PF_THREADS = 256;  // 4 waves
constexpr int PF_WAVES = PF_THREADS / 64;

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct PfGemmArgs {
    const void* w;     // [rows][K]
    size_t row_bytes;
    int K;
    int rows;
    const float* x;    // [n][K] f32
    int n;             // tokens in this pass (1..PF_TOK)
    int ks;            // K slices (K % (ks * 2E) == 0, host-checked)
    float* part;       // [ks][n][rows]
};

// PIPE: K slice a multiple of 4 chunk pairs (weights requested 4 pairs ahead).  RT: 32-row
// tiles per wave; each X operand load feeds RT x 2 accumulator tiles.
// gguf blocks (Q8_0 / Q4_0): each lane's 16-B chunk lies in one 32-element block; its f16 d
// (the planar row's scale area) multiplies the decoded codes, w = q * d exact in f32 as
// quants.py's dequantize (oracle xo_gq_elem), before the MFMA.
template <int DT, bool PIPE, int RT>
__global__ __launch_bounds__(PF_THREADS) void prefill_gemm_kernel(const PfGemmArgs a) {
    constexpr int E = WDec<DT>::E;
    constexpr bool GQ = gq_dt(DT);
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * PF_WAVES + (threadIdx.x >> 6);
    const int n_rt = (a.rows + 32 * RT - 1) / (32 * RT);
    if (gw >= n_rt * a.ks) return;
    const int rt = gw / a.ks, s = gw - rt * a.ks;
    const int j = lane & 31, h = lane >> 5;
    const int kslice = a.K / a.ks;
    const int k0 = s * kslice, k1 = k0 + kslice;
    const char* wrow[RT];
#pragma unroll
    for (int i = 0; i < RT; i++)
        wrow[i] = (const char*)a.w + (size_t)min((rt * RT + i) * 32 + j, a.rows - 1) * a.row_bytes;
    const int n_tt = (a.n + 31) / 32;
    // token rows of this lane's A operand in each tile (clamped: rows past n are not stored)
    const float* x0 = a.x + (size_t)min(j, a.n - 1) * a.K;
    const float* x1 = a.x + (size_t)min(32 + j, a.n - 1) * a.K;
    f32x16 acc0[RT], acc1[RT];
#pragma unroll
    for (int i = 0; i < RT; i++) acc0[i] = acc1[i] = f32x16{};
    // software pipeline over chunk pairs: (weights, X) of later pairs in flight while this
    // one's 2 E RT MFMAs run (weights come from HBM, X from L2)
    struct Stage {
        u32x4 w[RT];
        float d[RT];
        float4 x0[E / 4], x1[E / 4];
    };
    const size_t qb = GQ ? gq_qbytes(DT, (size_t)a.K) : 0;
    auto load = [&](Stage& st, const int kb) {
        const int k = kb + E * h;
#pragma unroll
        for (int i = 0; i < RT; i++) {
            st.w[i] = *(const u32x4*)(wrow[i] + (size_t)k * 16 / E);
            if constexpr (GQ) st.d[i] = f16_bits_to_f32(*(const uint16_t*)(wrow[i] + qb + (size_t)(k >> 5) * 2));
        }
#pragma unroll
        for (int q = 0; q < E / 4; q++) st.x0[q] = *(const float4*)(x0 + k + 4 * q);
        if (n_tt > 1) {
#pragma unroll
            for (int q = 0; q < E / 4; q++) st.x1[q] = *(const float4*)(x1 + k + 4 * q);
        }
    };
    auto mfma = [&](const Stage& st) {
#pragma unroll
        for (int i = 0; i < RT; i++) {
            float wf[E];
            WDec<DT>::dec(st.w[i], wf);
            if constexpr (GQ) {
#pragma unroll
                for (int e = 0; e < E; e++) wf[e] *= st.d[i];
            }
#pragma unroll
            for (int q = 0; q < E / 4; q++) {
                acc0[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(st.x0[q].x, wf[4 * q + 0], acc0[i], 0, 0, 0);
                acc0[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(st.x0[q].y, wf[4 * q + 1], acc0[i], 0, 0, 0);
                acc0[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(st.x0[q].z, wf[4 * q + 2], acc0[i], 0, 0, 0);
                acc0[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(st.x0[q].w, wf[4 * q + 3], acc0[i], 0, 0, 0);
            }
            if (n_tt > 1) {
#pragma unroll
                for (int q = 0; q < E / 4; q++) {
                    acc1[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(st.x1[q].x, wf[4 * q + 0], acc1[i], 0, 0, 0);
                    acc1[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(st.x1[q].y, wf[4 * q + 1], acc1[i], 0, 0, 0);
                    acc1[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(st.x1[q].z, wf[4 * q + 2], acc1[i], 0, 0, 0);
                    acc1[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(st.x1[q].w, wf[4 * q + 3], acc1[i], 0, 0, 0);
                }
            }
        }
    };
    if (PIPE) {
        // 4-deep ring of (weights, X) chunk pairs: a wave's loads complete in issue order
        // (vmcnt), so X travels with its weights and waiting for chunk c leaves c+1..c+3 in
        // flight.  (k1 - k0) % (8E) == 0 (host-checked); indices clamped so every load is
        // unconditional (the last chunk is re-read past the end, unused)
        const int P = (k1 - k0) / (2 * E);
        auto ld = [&](Stage& st, const int c) { load(st, k0 + 2 * E * min(c, P - 1)); };
        Stage s0, s1, s2, s3;
        ld(s0, 0);
        ld(s1, 1);
        ld(s2, 2);
        ld(s3, 3);
        for (int c = 0; c < P; c += 4) {
            mfma(s0);
            ld(s0, c + 4);
            mfma(s1);
            ld(s1, c + 5);
            mfma(s2);
            ld(s2, c + 6);
            mfma(s3);
            ld(s3, c + 7);
        }
    } else {
        Stage sa, sb;
        int kb = k0;
        load(sa, kb);
        for (; kb + 4 * E <= k1; kb += 4 * E) {
            load(sb, kb + 2 * E);
            mfma(sa);
            if (kb + 4 * E < k1) load(sa, kb + 4 * E);
            mfma(sb);
        }
        if (kb < k1) mfma(sa);  // odd count of chunk pairs: the last one, loaded above
    }
    // D map: column j = lane & 31 (row r), row i = (reg & 3) + 8 (reg >> 2) + 4 h (token)
#pragma unroll
    for (int i = 0; i < RT; i++) {
        const int r = (rt * RT + i) * 32 + j;
        if (r >= a.rows) continue;
        float* out = a.part + (size_t)s * a.n * a.rows + r;
#pragma unroll
        for (int reg = 0; reg < 16; reg++) {
            const int t = (reg & 3) + 8 * (reg >> 2) + 4 * h;
            if (t < a.n) out[(size_t)t * a.rows] = acc0[i][reg];
            if (n_tt > 1 && 32 + t < a.n) out[(size_t)(32 + t) * a.rows] = acc1[i][reg];
        }
    }
}

// ---- split-f16 GEMM (XH_OPT_PREFILL 2) ----------------------------------------------------
// Y = X W^T on v_mfma_f32_32x32x16_f16 (8x the K of the f32 MFMA per instruction, half its
// cycles).  Each activation row is scaled by a power of two s_t (row max in [2^14, 2^15)) and
// split exactly-as-possible into two f16: hi = f16(s x), lo = f16(s x - hi), |x - (hi+lo)/s|
// <= 2^-22 |x| (below f16's subnormal floor: 2^-38 of the row max).  Products are exact
// (f16 x f16 in f32) and accumulate in f32; the store multiplies by 1/s_t (exact).  Weights
// must convert exactly to f16: f16 itself, e4m3 (via f32), e5m2 (its code is an f16's top
// byte); bf16 / f32 / Q8 / NaN-holding fp8 take the f32-MFMA kernel.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// A-operand fragment layout of X for weights with E elements per 16 bytes (M = E / 8 MFMAs per
// chunk): block (token tile tt, chunk c of 2E k, m) holds 64 x 16 bytes, lane l's 8 f16 at
// 16 l = X[32 tt + (l & 31)][2E c + E (l >> 5) + 8 m + j], so a wave's fragment load is one
// contiguous 1 KB read (a row-major gather touches 32 rows per load and saturated L1).
__host__ __device__ inline size_t frag_off(const int tt, const int c, const int m, const int lane, const int n_c,
                                           const int M) {
    return ((((size_t)tt * n_c + c) * M + m) * 64 + lane) * 8;  // in f16 elements
}
// offset (f16 elements) of X[t][k .. k+8) in the split layout: E > 0 the fragment layout above,
// E == 0 plain row-major [t][K] (the hipBLASLt GEMM's B operand)
__device__ __forceinline__ size_t split_off(const int t, const int k, const int K, const int E) {
    if (E == 0) return (size_t)t * K + k;
    const int M = E / 8, n_c = K / (2 * E);
    const int c = k / (2 * E), r = k - c * 2 * E, hh = r / E, m = (r - hh * E) / 8;
    return frag_off(t >> 5, c, m, (t & 31) + 32 * hh, n_c, M);
}

// one workgroup per token row (grid = 32 x token tiles; rows past n are zero): s_t, hi, lo in
// the fragment layout, inv_s[t] = 1 / s_t
__global__ __launch_bounds__(256) void prefill_split_kernel(const float* x, int K, int n, int E, uint16_t* xh,
                                                            uint16_t* xl, float* inv_s) {
    __shared__ float red[4];
    const int t = blockIdx.x;
    if (t >= n) {
        for (int i = threadIdx.x; i < K / 8; i += 256) {
            const size_t o = split_off(t, 8 * i, K, E);
            *(u32x4*)(xh + o) = u32x4{0u, 0u, 0u, 0u};
            *(u32x4*)(xl + o) = u32x4{0u, 0u, 0u, 0u};
        }
        return;
    }
    const float* xr = x + (size_t)t * K;
    float m = 0.f;
    for (int i = threadIdx.x; i < K; i += 256) m = fmaxf(m, fabsf(xr[i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    // m = f 2^e with f in [0.5, 1): s = 2^(15 - e) puts s m in [2^14, 2^15); a zero or
    // non-finite row keeps s = 1
    int e = 0;
    const bool ok = m > 0.f && m <= FLT_MAX;
    if (ok) frexpf(m, &e);  // m = f * 2^e, f in [0.5, 1)
    const float s = ok ? ldexpf(1.f, 15 - e) : 1.f;
    for (int i = threadIdx.x; i < K / 8; i += 256) {
        const int k = 8 * i;
        const float4 a = *(const float4*)(xr + k), b = *(const float4*)(xr + k + 4);
        const float v[8] = {a.x * s, a.y * s, a.z * s, a.w * s, b.x * s, b.y * s, b.z * s, b.w * s};
        f16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            hi[j] = (_Float16)v[j];
            lo[j] = (_Float16)(v[j] - (float)hi[j]);
        }
        const size_t o = split_off(t, k, K, E);
        *(f16x8*)(xh + o) = hi;
        *(f16x8*)(xl + o) = lo;
    }
    if (threadIdx.x == 0) inv_s[t] = 1.f / s;
}

// rmsnorm of each token row (as prefill_rmsnorm_kernel: x * scale * w, same reduction) written
// straight into the split-f16 fragment layout for the GEMM that consumes it: one launch instead
// of rmsnorm + split (grid = 32 x token tiles; rows past n are zero)
__global__ __launch_bounds__(256) void prefill_rmsnorm_split_kernel(const float* x, int dim, const void* w, int wdt,
                                                                    float eps, int n, int E, uint16_t* xh,
                                                                    uint16_t* xl, float* inv_s) {
    __shared__ float red[4];
    const int t = blockIdx.x;
    auto frag = [&](const int k) { return split_off(t, k, dim, E); };
    if (t >= n) {
        for (int i = threadIdx.x; i < dim / 8; i += 256) {
            const size_t o = frag(8 * i);
            *(u32x4*)(xh + o) = u32x4{0u, 0u, 0u, 0u};
            *(u32x4*)(xl + o) = u32x4{0u, 0u, 0u, 0u};
        }
        return;
    }
    const float* xr = x + (size_t)t * dim;
    const float scale = block_rms_scale<256>(xr, dim, eps, red);
    __syncthreads();  // red reused below
    auto norm8 = [&](const int i, float* v) {  // elements 8i .. 8i+7 of the normed row
        const float4 a = ((const float4*)xr)[2 * i], b = ((const float4*)xr)[2 * i + 1];
        const float4 wa = load_norm4(w, wdt, 2 * i), wb = load_norm4(w, wdt, 2 * i + 1);
        v[0] = a.x * scale * wa.x; v[1] = a.y * scale * wa.y; v[2] = a.z * scale * wa.z; v[3] = a.w * scale * wa.w;
        v[4] = b.x * scale * wb.x; v[5] = b.y * scale * wb.y; v[6] = b.z * scale * wb.z; v[7] = b.w * scale * wb.w;
    };
    float m = 0.f;
    for (int i = threadIdx.x; i < dim / 8; i += 256) {
        float v[8];
        norm8(i, v);
#pragma unroll
        for (int j = 0; j < 8; j++) m = fmaxf(m, fabsf(v[j]));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    int e = 0;
    const bool ok = m > 0.f && m <= FLT_MAX;
    if (ok) frexpf(m, &e);
    const float s = ok ? ldexpf(1.f, 15 - e) : 1.f;
    for (int i = threadIdx.x; i < dim / 8; i += 256) {
        float v[8];
        norm8(i, v);
        f16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float u = v[j] * s;
            hi[j] = (_Float16)u;
            lo[j] = (_Float16)(u - (float)hi[j]);
        }
        const size_t o = frag(8 * i);
        *(f16x8*)(xh + o) = hi;
        *(f16x8*)(xl + o) = lo;
    }
    if (threadIdx.x == 0) inv_s[t] = 1.f / s;
}

// EPI_RESID of a GEMM's partials (x += the summed K-slices, slice order, times part_s, as
// prefill_epi_kernel) and the rmsnorm split of the updated row for the next GEMM (as
// prefill_rmsnorm_split_kernel: the same per-thread float4 order, reduction and split), in one
// launch: the residual row is read once.  part_s and inv_s may both be pf_xs: a workgroup reads
// its token's factor before the first barrier and writes the new one after the last.  Dynamic
// LDS: the updated row (dim floats).  grid = 32 x token tiles; rows past n are zero.
__global__ __launch_bounds__(256) void prefill_resid_norm_split_kernel(const float* part, int ks, const float* part_s,
                                                                       float* x, int dim, const void* w, int wdt,
                                                                       float eps, int n, int E, uint16_t* xh,
                                                                       uint16_t* xl, float* inv_s) {
    extern __shared__ __attribute__((aligned(16))) float xrow[];  // float4 reads and writes
    __shared__ float red[4];
    const int t = blockIdx.x;
    auto frag = [&](const int k) { return split_off(t, k, dim, E); };
    if (t >= n) {
        for (int i = threadIdx.x; i < dim / 8; i += 256) {
            const size_t o = frag(8 * i);
            *(u32x4*)(xh + o) = u32x4{0u, 0u, 0u, 0u};
            *(u32x4*)(xl + o) = u32x4{0u, 0u, 0u, 0u};
        }
        return;
    }
    float4* xr4 = (float4*)(x + (size_t)t * dim);
    const float ps = part_s ? part_s[t] : 1.f;
    float ss = 0.f;
    for (int i = threadIdx.x; i < (dim >> 2); i += 256) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s = 0; s < ks; s++) {  // slice order: fixed
            const float4 p = *(const float4*)(part + ((size_t)s * n + t) * dim + 4 * i);
            v.x += p.x;
            v.y += p.y;
            v.z += p.z;
            v.w += p.w;
        }
        if (part_s) {
            v.x *= ps;
            v.y *= ps;
            v.z *= ps;
            v.w *= ps;
        }
        float4 r = xr4[i];
        r.x += v.x;
        r.y += v.y;
        r.z += v.z;
        r.w += v.w;
        xr4[i] = r;
        ((float4*)xrow)[i] = r;
        ss += r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w;
    }
    // block_rms_scale<256>'s reduction
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; wv++) tot += red[wv];
    const float rms = sqrtf(tot / (float)dim + eps);
    const float scale = 1.0f / rms;
    __syncthreads();  // red reused below
    auto norm8 = [&](const int i, float* v) {  // elements 8i .. 8i+7 of the normed row
        const float4 a = ((const float4*)xrow)[2 * i], b = ((const float4*)xrow)[2 * i + 1];
        const float4 wa = load_norm4(w, wdt, 2 * i), wb = load_norm4(w, wdt, 2 * i + 1);
        v[0] = a.x * scale * wa.x; v[1] = a.y * scale * wa.y; v[2] = a.z * scale * wa.z; v[3] = a.w * scale * wa.w;
        v[4] = b.x * scale * wb.x; v[5] = b.y * scale * wb.y; v[6] = b.z * scale * wb.z; v[7] = b.w * scale * wb.w;
    };
    float m = 0.f;
    for (int i = threadIdx.x; i < dim / 8; i += 256) {
        float v[8];
        norm8(i, v);
#pragma unroll
        for (int j = 0; j < 8; j++) m = fmaxf(m, fabsf(v[j]));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    int e = 0;
    const bool ok = m > 0.f && m <= FLT_MAX;
    if (ok) frexpf(m, &e);
    const float s = ok ? ldexpf(1.f, 15 - e) : 1.f;
    for (int i = threadIdx.x; i < dim / 8; i += 256) {
        float v[8];
        norm8(i, v);
        f16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float u = v[j] * s;
            hi[j] = (_Float16)u;
            lo[j] = (_Float16)(u - (float)hi[j]);
        }
        const size_t o = frag(8 * i);
        *(f16x8*)(xh + o) = hi;
        *(f16x8*)(xl + o) = lo;
    }
    if (threadIdx.x == 0) inv_s[t] = 1.f / s;
}

// EPI_GLU (act(g) * u of the summed K-slices, slice order as prefill_epi_kernel) written
// straight into the split-f16 fragments of the W2 GEMM's input: one launch instead of GLU
// epilogue + split.  The row (hidden f32) is held in dynamic LDS between the max and the split
// (grid = 32 x token tiles; rows past n are zero)
// part_s (nullable): per-token factor of the partials (the hipBLASLt GEMM's 1 / s of its input)
__global__ __launch_bounds__(1024) void prefill_glu_split_kernel(const float* part, int ks, int n, int hidden, int act,
                                                                int E, uint16_t* xh, uint16_t* xl, float* inv_s,
                                                                const float* part_s) {
    extern __shared__ float hrow[];
    __shared__ float red[16];
    const int t = blockIdx.x;
    auto frag = [&](const int k) { return split_off(t, k, hidden, E); };
    if (t >= n) {
        for (int i = threadIdx.x; i < hidden / 8; i += 1024) {
            const size_t o = frag(8 * i);
            *(u32x4*)(xh + o) = u32x4{0u, 0u, 0u, 0u};
            *(u32x4*)(xl + o) = u32x4{0u, 0u, 0u, 0u};
        }
        return;
    }
    const size_t rows = 2 * (size_t)hidden;
    float m = 0.f;
    // two (g, u) pairs per 16-byte load (hidden % 32 == 0 on the batched path): 73.6 -> 53.9 us per
    // 2048-token launch against one pair per 8-byte load (rocprof, same box)
    const float ps = part_s ? part_s[t] : 1.f;
#pragma unroll 4
    for (int i = threadIdx.x; i < (hidden >> 1); i += 1024) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s = 0; s < ks; s++) {  // slice order: fixed
            const float4 p = *(const float4*)(part + ((size_t)s * n + t) * rows + 4 * i);
            v.x += p.x;
            v.y += p.y;
            v.z += p.z;
            v.w += p.w;
        }
        if (part_s) {
            v.x *= ps;
            v.y *= ps;
            v.z *= ps;
            v.w *= ps;
        }
        const float h0 = act_fn(act, v.x) * v.y, h1 = act_fn(act, v.z) * v.w;
        hrow[2 * i] = h0;
        hrow[2 * i + 1] = h1;
        m = fmaxf(m, fmaxf(fabsf(h0), fabsf(h1)));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = red[0];
    for (int w = 1; w < 16; w++) m = fmaxf(m, red[w]);
    int e = 0;
    const bool ok = m > 0.f && m <= FLT_MAX;
    if (ok) frexpf(m, &e);
    const float s = ok ? ldexpf(1.f, 15 - e) : 1.f;
    for (int i = threadIdx.x; i < hidden / 8; i += 1024) {
        f16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float u = hrow[8 * i + j] * s;
            hi[j] = (_Float16)u;
            lo[j] = (_Float16)(u - (float)hi[j]);
        }
        const size_t o = frag(8 * i);
        *(f16x8*)(xh + o) = hi;
        *(f16x8*)(xl + o) = lo;
    }
    if (threadIdx.x == 0) inv_s[t] = 1.f / s;
}

// 16 weight bytes -> E/8 B operands of 8 f16 (k order = byte order)
template <int DT>
__device__ __forceinline__ void w_f16(const u32x4 w, f16x8* b) {
    if constexpr (DT == XH_F16) {
        b[0] = __builtin_bit_cast(f16x8, w);
    } else if constexpr (DT == XH_F8_E5M2) {
        const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int e = 0; e < 16; e++)  // code c -> f16 bits c << 8
            b[e >> 3][e & 7] = __builtin_bit_cast(_Float16, (uint16_t)(((u[e >> 2] >> (8 * (e & 3))) & 0xffu) << 8));
    } else {
        static_assert(DT == XH_F8_E4M3, "split-f16 GEMM: weights must convert exactly to f16");
        float f[16];
        WDec<DT>::dec(w, f);
#pragma unroll
        for (int e = 0; e < 16; e++) b[e >> 3][e & 7] = (_Float16)f[e];  // exact: e4m3 fits f16
    }
}

struct PfGemm16Args {
    const void* w;        // [rows][K]
    size_t row_bytes;
    int K, rows;
    const uint16_t* xh;   // [n][K] f16 bits
    const uint16_t* xl;
    const float* inv_s;   // [n]
    int n, ks;
    float* part;          // [ks][n][rows]
};

// Lane l of a wave: weight bytes of row (tile i, l & 31) at k = kb + E h (h = l >> 5); MFMA
// m of the chunk pairs B = 8 of them (k = kb + E h + 8 m + j) with A = X at the same k, so
// A and B agree on k for every lane (the sum over k is order-free up to f32 rounding).
template <int DT, int RT>
__global__ __launch_bounds__(PF_THREADS) void prefill_gemm16_kernel(const PfGemm16Args a) {
    constexpr int E = WDec<DT>::E;
    constexpr int ESZ = 16 / E;
    constexpr int M = E / 8;  // MFMAs per 16 weight bytes
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * PF_WAVES + (threadIdx.x >> 6);
    const int n_rt = (a.rows + 32 * RT - 1) / (32 * RT);
    if (gw >= n_rt * a.ks) return;
    const int rt = gw / a.ks, s = gw - rt * a.ks;
    const int j = lane & 31, h = lane >> 5;
    const int kslice = a.K / a.ks;
    const int k0 = s * kslice;
    const char* wrow[RT];
#pragma unroll
    for (int i = 0; i < RT; i++)
        wrow[i] = (const char*)a.w + (size_t)min((rt * RT + i) * 32 + j, a.rows - 1) * a.row_bytes;
    const int n_tt = (a.n + 31) / 32;
    const int n_c = a.K / (2 * E);
    f32x16 acc0[RT], acc1[RT];
#pragma unroll
    for (int i = 0; i < RT; i++) acc0[i] = acc1[i] = f32x16{};
    struct Stage {
        u32x4 w[RT];
        u32x4 h0[M], l0[M], h1[M], l1[M];
    };
    // chunk c: weights at k = 2E c + E h; X fragments of token tiles 0 / 1 (prefill_split_kernel)
    auto load = [&](Stage& st, const int c) {
        const int k = 2 * E * c + E * h;
#pragma unroll
        for (int i = 0; i < RT; i++) st.w[i] = *(const u32x4*)(wrow[i] + (size_t)k * ESZ);
#pragma unroll
        for (int m = 0; m < M; m++) {
            st.h0[m] = *(const u32x4*)(a.xh + frag_off(0, c, m, lane, n_c, M));
            st.l0[m] = *(const u32x4*)(a.xl + frag_off(0, c, m, lane, n_c, M));
        }
        if (n_tt > 1) {
#pragma unroll
            for (int m = 0; m < M; m++) {
                st.h1[m] = *(const u32x4*)(a.xh + frag_off(1, c, m, lane, n_c, M));
                st.l1[m] = *(const u32x4*)(a.xl + frag_off(1, c, m, lane, n_c, M));
            }
        }
    };
    auto mfma = [&](const Stage& st) {
#pragma unroll
        for (int i = 0; i < RT; i++) {
            f16x8 b[M];
            w_f16<DT>(st.w[i], b);
#pragma unroll
            for (int m = 0; m < M; m++) {
                acc0[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, st.h0[m]), b[m], acc0[i], 0, 0, 0);
                acc0[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, st.l0[m]), b[m], acc0[i], 0, 0, 0);
            }
            if (n_tt > 1) {
#pragma unroll
                for (int m = 0; m < M; m++) {
                    acc1[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, st.h1[m]), b[m], acc1[i], 0, 0, 0);
                    acc1[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, st.l1[m]), b[m], acc1[i], 0, 0, 0);
                }
            }
        }
    };
    // 4-deep ring over chunk pairs (2E k per stage); kslice % (8E) == 0 (host-checked);
    // clamped indices keep every load unconditional
    const int P = kslice / (2 * E);
    auto ld = [&](Stage& st, const int c) { load(st, k0 / (2 * E) + min(c, P - 1)); };
    Stage s0, s1, s2, s3;
    ld(s0, 0);
    ld(s1, 1);
    ld(s2, 2);
    ld(s3, 3);
    for (int c = 0; c < P; c += 4) {
        mfma(s0);
        ld(s0, c + 4);
        mfma(s1);
        ld(s1, c + 5);
        mfma(s2);
        ld(s2, c + 6);
        mfma(s3);
        ld(s3, c + 7);
    }
    // D map: column j = lane & 31 (row r), row i = (reg & 3) + 8 (reg >> 2) + 4 h (token)
#pragma unroll
    for (int i = 0; i < RT; i++) {
        const int r = (rt * RT + i) * 32 + j;
        if (r >= a.rows) continue;
        float* out = a.part + (size_t)s * a.n * a.rows + r;
#pragma unroll
        for (int reg = 0; reg < 16; reg++) {
            const int t = (reg & 3) + 8 * (reg >> 2) + 4 * h;
            if (t < a.n) out[(size_t)t * a.rows] = acc0[i][reg] * a.inv_s[t];
            if (n_tt > 1 && 32 + t < a.n) out[(size_t)(32 + t) * a.rows] = acc1[i][reg] * a.inv_s[32 + t];
        }
    }
}

// Per-pass token scalars
struct PfEpiArgs {
    const float* part;  // [ks][n][rows]
    const float* part_s;  // nullable: [n] factor of token t's summed partials (hipBLASLt: 1 / s_t)
    int ks, n, rows;
    int epi;            // EPI_QKV / EPI_RESID / EPI_GLU / EPI_STORE
    float* out;         // RESID: X [n][rows] (+=); GLU: H [n][rows/2]; STORE: [n][out_stride]
    size_t out_stride;  // STORE row stride (0: rows)
    // EPI_QKV
    float* q;           // [n][q_dim]
    uint16_t* kcache;   // this layer's rings [max_seq_len][kv_dim]
    uint16_t* vcache;
    int q_dim, kv_dim, head_dim;
    const float* rope_freq;
    float qkv_clip;
    int pos0;           // position of token 0 of the pass (ring slot = pos, no wrap in a pass)
    int act;
};

__global__ __launch_bounds__(256) void prefill_epi_kernel(const PfEpiArgs a) {
    // one thread per output pair (rows are even for QKV / GLU / RESID; STORE may be odd: the
    // last pair's second row is not written)
    const int pairs = (a.rows + 1) / 2;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.n * pairs) return;
    const int t = idx / pairs, r = 2 * (idx - t * pairs);
    float v0 = 0.f, v1 = 0.f;
    const bool two = r + 1 < a.rows;
    for (int s = 0; s < a.ks; s++) {  // slice order: fixed
        const float* p = a.part + ((size_t)s * a.n + t) * a.rows + r;
        v0 += p[0];
        if (two) v1 += p[1];
    }
    if (a.part_s) {
        v0 *= a.part_s[t];
        v1 *= a.part_s[t];
    }
    if (a.epi == EPI_RESID) {
        float* o = a.out + (size_t)t * a.rows + r;
        o[0] += v0;
        o[1] += v1;
    } else if (a.epi == EPI_STORE) {
        float* o = a.out + (size_t)t * (a.out_stride ? a.out_stride : a.rows) + r;
        o[0] = v0;
        if (r + 1 < a.rows) o[1] = v1;
    } else if (a.epi == EPI_GLU) {
        a.out[(size_t)t * (a.rows / 2) + r / 2] = act_fn(a.act, v0) * v1;
    } else {  // EPI_QKV: src/infer.cpp:392-414 at pos = pos0 + t
        const int pos = a.pos0 + t;
        v0 = clipf(v0, a.qkv_clip);
        v1 = clipf(v1, a.qkv_clip);
        if (r < a.q_dim) {
            rope_pair(v0, v1, r, a.head_dim, pos, a.rope_freq);
            a.q[(size_t)t * a.q_dim + r] = v0;
            a.q[(size_t)t * a.q_dim + r + 1] = v1;
        } else {
            const bool isk = r < a.q_dim + a.kv_dim;
            const int kr = isk ? r - a.q_dim : r - a.q_dim - a.kv_dim;
            if (isk) rope_pair(v0, v1, kr, a.head_dim, pos, a.rope_freq);
            uint16_t* dst = (isk ? a.kcache : a.vcache) + (size_t)pos * a.kv_dim + kr;
            *(uint32_t*)dst = (uint32_t)f32_to_f16_bits(v0) | ((uint32_t)f32_to_f16_bits(v1) << 16);
        }
    }
}

// rmsnorm of each token row (src/infer.cpp:224-236), one workgroup per token; same reduction
// shape as block_rms_scale
__global__ __launch_bounds__(256) void prefill_rmsnorm_kernel(const float* x, int dim, const void* w, int wdt,
                                                              float eps, float* o) {
    __shared__ float red[4];
    const float* xr = x + (size_t)blockIdx.x * dim;
    const float scale = block_rms_scale<256>(xr, dim, eps, red);
    float* orow = o + (size_t)blockIdx.x * dim;
    for (int i = threadIdx.x; i < (dim >> 2); i += 256) {
        const float4 v = ((const float4*)xr)[i];
        const float4 ww = load_norm4(w, wdt, i);
        ((float4*)orow)[i] = make_float4(v.x * scale * ww.x, v.y * scale * ww.y, v.z * scale * ww.z, v.w * scale * ww.w);
    }
}

// x rows of the pass = embedding rows of the tokens (Model::_copy_embedding)
__global__ __launch_bounds__(256) void prefill_embed_kernel(const int* tokens, const void* emb, int dtype, int dim,
                                                            float* x) {
    const size_t row = (size_t)tokens[blockIdx.x];
    for (int i = threadIdx.x; i < dim; i += 256) x[(size_t)blockIdx.x * dim + i] = dec_row(dtype, emb, row, dim, i);
}

// attention of the pass's tokens: grid (n_kv_heads, nsplit, n); token t attends to slots
// [0, pos0 + t] (its own K/V row included), per-token StepParams in sps[t]
template <int HD, int QPK>
__global__ __launch_bounds__(ATTN_THREADS) void prefill_attn_kernel(AttnArgs a, const StepParams* sps, int q_stride,
                                                                    int n_kv_heads) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = blockIdx.z;
    a.q += (size_t)t * q_stride;
    a.out += (size_t)t * q_stride;
    a.part_o += (size_t)t * a.nsplit * q_stride;
    a.part_ml += (size_t)t * a.nsplit * a.n_heads * 2;
    a.counters += t * n_kv_heads;
    a.sp = sps + t;
    attn_block<HD, QPK, ATTN_THREADS, false>(a, blockIdx.x, blockIdx.y, smem, nullptr);
}

// One 32-slot tile of the prompt attention's online softmax (both kernels below): scores
// s = st * (1 / row scale) * (1/sqrtf(hd)) (the first factor a power of two: one rounding), masked
// past each row's pos on the diagonal tiles only (diag: wave-uniform), running max m over the
// lane pair (l, l ^ 32), p = e^(s - m) split into exact f16 hi + lo (|p - hi - lo| <= 2^-25), O and
// the running sum rescaled by e^(m_old - m) — skipped when it is 1 in every lane (exact: x * 1 = x).
// e^x by v_exp_f32 of x log2(e) (__expf: <= 2e-6 relative at the x > -20 that carry weight).
template <int NDT>
__device__ __forceinline__ void fa_softmax_tile(const f32x16& st, const int b, const int pos, const int h,
                                                const float sc, const bool diag, float& m, float& lsum,
                                                f32x16 (&o)[NDT], f16x8 (&ph)[2], f16x8 (&pl)[2]) {
    float sv[16];
    float tm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        float v = st[r] * sc;
        if (diag) v = b + (r & 3) + 8 * (r >> 2) + 4 * h <= pos ? v : -INFINITY;
        sv[r] = v;
        tm = fmaxf(tm, v);
    }
    tm = fmaxf(tm, __shfl_xor(tm, 32));
    const float mn = fmaxf(m, tm);  // finite: slot 0 <= pos on the first tile
    const float alpha = __expf(m - mn);
    m = mn;
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const float p = __expf(sv[r] - mn);
        ps += p;
        const _Float16 hi = (_Float16)p;
        ph[r >> 3][r & 7] = hi;
        pl[r >> 3][r & 7] = (_Float16)(p - (float)hi);
    }
    lsum = lsum * alpha + ps;
    if (!__all(alpha == 1.f)) {
#pragma unroll
        for (int dt = 0; dt < NDT; dt++) o[dt] *= alpha;
    }
}

// ---- causal attention of a prompt pass on MFMA ------------------------------------------
// Per token and head (src/infer.cpp:279-301 / :338): s_t = (q . K[t]) * (1/sqrtf(hd)) over slots
// [0, pos], p = softmax(s) (max-subtract, expf), out = sum_t p_t V[t].  Computed flash-style
// over 32-slot tiles with a running max and sum (f32), the sum divided out at the end.
// One wave = one KV head x 32 query rows (32/QPK tokens x the QPK heads sharing that KV head).
//   S^T = K Q^T on v_mfma_f32_32x32x16_f16: A = K rows (exact f16), B = q split into exact
//         f16 hi + lo under a power-of-two row scale (as prefill_split_kernel; <= 2^-22 |q|),
//         two MFMAs per 16-wide k step, products exact in f32.  D: lane (h, row j) holds the
//         16 slots (r & 3) + 8 (r >> 2) + 4 h of query row j, so the row's max / sum is one
//         lane pair (l, l ^ 32) and the rescale of O is a per-lane scalar.
//   O^T = V^T P^T: B = p (this lane's own 16 values, as f16 hi + lo: |p - hi - lo| <= 2^-25),
//         A = V^T fragments from a transposed LDS copy of the V tile; the k index of MFMA step
//         s, lane half h, element e is slot 16 s + 8 (e >> 2) + 4 h + (e & 3) on both sides.
// grid (n_kv_heads, ceil(n / (32/QPK))), 64 threads; no ring wrap inside a pass (pf_supported)
template <int HD, int QPK>
__global__ __launch_bounds__(64) void prefill_fa_kernel(const float* q, const uint16_t* kc, const uint16_t* vc,
                                                         float* out, int n, int pos0, int q_stride, int kv_dim) {
    constexpr int TPW = 32 / QPK;        // tokens per wave
    constexpr int KS = HD / 16;          // k steps of q . k
    constexpr int NDT = (HD + 31) / 32;  // 32-row d tiles of O^T
    constexpr int VP = 40;               // V^T row pitch (f16): conflict-free 8-byte fragment reads
    static_assert(HD % 16 == 0 && 32 % QPK == 0, "prefill_fa_kernel: head shape");
    __shared__ __attribute__((aligned(16))) uint16_t vt[NDT * 32 * VP];
    const int lane = threadIdx.x, j32 = lane & 31, h = lane >> 5;
    const int g = blockIdx.x;
    const int t0 = (gridDim.y - 1 - blockIdx.y) * TPW;  // longest rows first
    const int tq = t0 + j32 / QPK;
    const int tqc = min(tq, n - 1);
    const int pos = pos0 + tqc;
    const int head = g * QPK + j32 % QPK;
    const int last = pos0 + min(t0 + TPW, n) - 1;  // the wave's last slot
    const float scale = 1.0f / sqrtf((float)HD);  // src/infer.cpp:338
    // q row, split: this lane's k = 16 ks + 8 h + e
    f16x8 qh[KS], ql[KS];
    float inv_s;
    {
        const float* qr = q + (size_t)tqc * q_stride + (size_t)head * HD;
        float v[KS][8];
        float mx = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            const float4 a = *(const float4*)(qr + 16 * ks + 8 * h), b = *(const float4*)(qr + 16 * ks + 8 * h + 4);
            v[ks][0] = a.x; v[ks][1] = a.y; v[ks][2] = a.z; v[ks][3] = a.w;
            v[ks][4] = b.x; v[ks][5] = b.y; v[ks][6] = b.z; v[ks][7] = b.w;
#pragma unroll
            for (int e = 0; e < 8; e++) mx = fmaxf(mx, fabsf(v[ks][e]));
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        int ex = 0;
        const bool ok = mx > 0.f && mx <= FLT_MAX;
        if (ok) frexpf(mx, &ex);
        const float sc = ok ? ldexpf(1.f, 15 - ex) : 1.f;
        inv_s = 1.f / sc;
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const float u = v[ks][e] * sc;
                qh[ks][e] = (_Float16)u;
                ql[ks][e] = (_Float16)(u - (float)qh[ks][e]);
            }
    }
    if (HD < 32) {  // rows d >= HD of the single d tile read as zero
        for (int i = lane; i < (32 - HD) * VP / 2; i += 64) ((uint32_t*)(vt + HD * VP))[i] = 0u;
    }
    f32x16 o[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; dt++) o[dt] = f32x16{};
    float m = -INFINITY, lsum = 0.f;
    const uint16_t* kg = kc + (size_t)g * HD;
    const uint16_t* vg = vc + (size_t)g * HD;
    constexpr int VCH = 16 * HD / 8;  // (slot pair, 8 d) chunks of a V tile
    constexpr int VIT = (VCH + 63) / 64;
    for (int b = 0; b <= last; b += 32) {
        // V tile -> registers (zeros past the wave's last slot: garbage x p = 0 could be NaN)
        u32x4 va[VIT], vb[VIT];
#pragma unroll
        for (int it = 0; it < VIT; it++) {
            const int c = lane + 64 * it, sp = c & 15, d8 = c >> 4;
            const int s0 = b + 2 * sp;
            va[it] = vb[it] = u32x4{0u, 0u, 0u, 0u};
            if (c < VCH) {
                if (s0 <= last) va[it] = *(const u32x4*)(vg + (size_t)s0 * kv_dim + 8 * d8);
                if (s0 + 1 <= last) vb[it] = *(const u32x4*)(vg + (size_t)(s0 + 1) * kv_dim + 8 * d8);
            }
        }
        // S^T = K Q^T (K rows clamped to the wave's range; masked below)
        f32x16 st = f32x16{};
        {
            const uint16_t* kr = kg + (size_t)min(b + j32, last) * kv_dim + 8 * h;
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                const f16x8 kf = __builtin_bit_cast(f16x8, *(const u32x4*)(kr + 16 * ks));
                st = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qh[ks], st, 0, 0, 0);
                st = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, ql[ks], st, 0, 0, 0);
            }
        }
        __syncthreads();  // the previous tile's V^T reads are done
#pragma unroll
        for (int it = 0; it < VIT; it++) {
            const int c = lane + 64 * it, sp = c & 15, d8 = c >> 4;
            if (c < VCH) {
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    const uint32_t lo = (va[it][e >> 1] >> (16 * (e & 1))) & 0xffffu;
                    const uint32_t hi = (vb[it][e >> 1] >> (16 * (e & 1))) & 0xffffu;
                    *(uint32_t*)(vt + (8 * d8 + e) * VP + 2 * sp) = lo | (hi << 16);
                }
            }
        }
        f16x8 ph[2], pl[2];
        fa_softmax_tile<NDT>(st, b, pos, h, inv_s * scale, b + 31 > pos0 + t0, m, lsum, o, ph, pl);
        __syncthreads();  // V^T tile written
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++) {
#pragma unroll
            for (int dt = 0; dt < NDT; dt++) {
                const uint16_t* vr = vt + (32 * dt + j32) * VP + 16 * s2 + 4 * h;
                const uint2 x0 = *(const uint2*)vr, x1 = *(const uint2*)(vr + 8);
                const f16x8 vf = __builtin_bit_cast(f16x8, u32x4{x0.x, x0.y, x1.x, x1.y});
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, ph[s2], o[dt], 0, 0, 0);
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pl[s2], o[dt], 0, 0, 0);
            }
        }
    }
    const float l = lsum + __shfl_xor(lsum, 32);
    if (tq >= n) return;
    const float inv_l = 1.f / l;
    float* orow = out + (size_t)tq * q_stride + (size_t)head * HD;
#pragma unroll
    for (int dt = 0; dt < NDT; dt++)
#pragma unroll
        for (int r = 0; r < 16; r += 4) {
            const int d = 32 * dt + 8 * (r >> 2) + 4 * h;
            if (d < HD)
                *(float4*)(orow + d) =
                    float4{o[dt][r] * inv_l, o[dt][r + 1] * inv_l, o[dt][r + 2] * inv_l, o[dt][r + 3] * inv_l};
        }
}

// ---- the same causal attention with K/V tiles shared by NW waves (head_dim 128) -------------
// prefill_fa_kernel's per-wave arithmetic, unchanged (same tiles, same MFMA order: the outputs
// are bit-identical), but a workgroup of NW waves covers NW x 32 query rows of one KV head and
// each 32-slot K / V tile goes L2 -> LDS ONCE for all of them, by global_load_lds_dwordx4, into a
// ring of FA_NS stages of FA_TPS tiles, issued FA_NS - 1 stages ahead of the multiply (counted
// vmcnt + raw s_barrier, as gemm16.h; two tiles per stage halve the barriers: +3.7 % at pos0 30719).  The single-wave kernel reads every K / V row once per wave from L2
// with its loads exposed (one round trip per tile); here a tile costs one DMA per NW waves and
// its latency hides under the previous tiles' MFMAs.
// LDS image of a tile ([32 slots][128 f16], 256-B rows): 16-B chunk c of row r at byte
// 256 r + 16 (c ^ (((r & 3) << 2) | ((r >> 2) & 3))) — one image serves the K row reads (S^T's
// A operand, ds_read_b128) and the V column reads (O^T's A operand = V^T, ds_read_b64_tr_b16:
// lane 4q+p of a 16-lane group gives row q, columns 4p..4p+3 of a 4 x 16 block and receives
// column (lane & 15) of the 4 rows), both conflict-free.  DMA writes are lane-linear, so the
// chunk permutation is applied to the per-lane source address.  Slots past the workgroup's last
// are clamped to it (valid rows; their p is 0 in every wave).
// a ring stage holds FA_TPS consecutive 32-slot K/V tiles (one counted wait + barrier per stage)
#ifndef PF_FA_TPS
#define PF_FA_TPS 2
#endif
constexpr int FA_TPS = PF_FA_TPS;
constexpr int FA_NS = FA_TPS >= 2 ? 2 : 3;  // ring stages
#ifndef PF_FA_ZIGZAG
#define PF_FA_ZIGZAG 1
#endif
#ifndef PF_FA_WAVES
#define PF_FA_WAVES 4                    // waves per workgroup
#endif
constexpr int FA_TILE_BYTES = 32 * 256;  // one K (or V) tile at head_dim 128
constexpr int FA_STAGE_BYTES = FA_TPS * 2 * FA_TILE_BYTES;
__host__ __device__ constexpr int fa_lds_bytes() { return FA_NS * FA_STAGE_BYTES; }
__device__ __forceinline__ uint32_t fa_off(const int r, const int c) {
    return (uint32_t)(256 * r + 16 * (c ^ (((r & 3) << 2) | ((r >> 2) & 3))));
}
typedef short fa_s16x4 __attribute__((ext_vector_type(4)));

// History split (grid z = nsplit > 1, a pass too short to fill the chip over a long history):
// workgroup z walks ring stages [z H / nsplit, (z + 1) H / nsplit) with H = pos0 / 64 (the last
// split runs to the workgroup's last slot), so every split starts at a slot <= pos0 <= each
// row's pos and its first tile has a finite max; it writes its unnormalised O and (m, l) to
// part_o [z][n][q_stride] / part_ml [z][n][n_heads], and prefill_fa_merge_kernel combines the
// splits in split order (deterministic).
template <int QPK, int NW>
__global__ __launch_bounds__(64 * NW, 2) void prefill_fa2_kernel(const float* q, const uint16_t* kc, const uint16_t* vc,
                                                               float* out, int n, int pos0, int q_stride, int kv_dim,
                                                               float* part_o, float2* part_ml) {
    constexpr int HD = 128;
    constexpr int TPW = 32 / QPK;        // tokens per wave
    constexpr int KS = HD / 16;          // k steps of q . k
    constexpr int NDT = HD / 32;         // 32-row d tiles of O^T
    constexpr int IPW = 16 * FA_TPS / NW;  // DMA wave-instructions per wave per stage (16 x 1 KiB per tile)
    static_assert(32 % QPK == 0 && (16 * FA_TPS) % NW == 0, "prefill_fa2_kernel: shape");
    extern __shared__ __attribute__((aligned(16))) char fa_smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int j32 = lane & 31, h = lane >> 5;
    const int g = blockIdx.x;
#if PF_FA_ZIGZAG
    // longest query tiles first, then the shortest first: with two workgroups per CU placed in
    // dispatch order (b and b + CUs), a CU's pair of causal tiles sums to the same length
    const int ny = gridDim.y, hy = (ny + 1) / 2, y = blockIdx.y;
    const int tb = (y < hy ? ny - 1 - y : y - hy) * (NW * TPW);
#else
    const int tb = (gridDim.y - 1 - blockIdx.y) * (NW * TPW);  // longest rows first
#endif
    const int t0 = tb + wv * TPW;                              // this wave's first token
    const int tq = t0 + j32 / QPK;
    const int tqc = min(tq, n - 1);
    const int pos = pos0 + tqc;
    const int head = g * QPK + j32 % QPK;
    const int last = t0 < n ? pos0 + min(t0 + TPW, n) - 1 : -1;  // this wave's last slot (-1: no rows)
    const int last_wg = pos0 + min(tb + NW * TPW, n) - 1;   // the workgroup's
    const float scale = 1.0f / sqrtf((float)HD);  // src/infer.cpp:338

    // DMA sources: instruction i of this wave = tile i >> 4 of the stage, image ((i >> 3) & 1: K, V),
    // rows 4 (i & 7) .. + 3
    int drow[IPW], dch[IPW];
#pragma unroll
    for (int k = 0; k < IPW; k++) {
        const int i = wv * IPW + k;
        drow[k] = 32 * (i >> 4) + 4 * (i & 7) + (lane >> 4);  // slot offset within the stage
        const int r = drow[k] & 31;
        dch[k] = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
    }
    const int ntile = last_wg / 32 + 1;
    const int nst_all = (ntile + FA_TPS - 1) / FA_TPS;
    const int nsplit = gridDim.z, z = blockIdx.z;
    const int hst = pos0 / (32 * FA_TPS);  // stage boundaries at or below pos0
    const int st0 = nsplit > 1 ? z * hst / nsplit : 0;
    const int nst = (nsplit > 1 && z < nsplit - 1 ? (z + 1) * hst / nsplit : nst_all) - st0;
    auto issue = [&](const int stage, const int st) {
        char* base = fa_smem + stage * FA_STAGE_BYTES;
#pragma unroll
        for (int k = 0; k < IPW; k++) {
            const int i = wv * IPW + k;
            const uint16_t* src = (((i >> 3) & 1) ? vc : kc) + (size_t)min(32 * FA_TPS * (st0 + st) + drow[k], last_wg) * kv_dim +
                                  (size_t)g * HD + 8 * dch[k];
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(base + i * 1024), 16, 0, 0);
        }
    };
    // q row, split: this lane's k = 16 ks + 8 h + e (loads before the ring's first DMA)
    f16x8 qh[KS], ql[KS];
    float inv_s;
    {
        const float* qr = q + (size_t)tqc * q_stride + (size_t)head * HD;
        float v[KS][8];
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            const float4 a = *(const float4*)(qr + 16 * ks + 8 * h), b = *(const float4*)(qr + 16 * ks + 8 * h + 4);
            v[ks][0] = a.x; v[ks][1] = a.y; v[ks][2] = a.z; v[ks][3] = a.w;
            v[ks][4] = b.x; v[ks][5] = b.y; v[ks][6] = b.z; v[ks][7] = b.w;
        }
        float mx = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
#pragma unroll
            for (int e = 0; e < 8; e++) mx = fmaxf(mx, fabsf(v[ks][e]));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        int ex = 0;
        const bool ok = mx > 0.f && mx <= FLT_MAX;
        if (ok) frexpf(mx, &ex);
        const float sc = ok ? ldexpf(1.f, 15 - ex) : 1.f;
        inv_s = 1.f / sc;
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const float u = v[ks][e] * sc;
                qh[ks][e] = (_Float16)u;
                ql[ks][e] = (_Float16)(u - (float)qh[ks][e]);
            }
    }
    mm_wait_vm<0>();
#pragma unroll
    for (int d = 0; d < FA_NS - 1; d++)
        if (d < nst) issue(d, d);

    f32x16 o[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; dt++) o[dt] = f32x16{};
    float m = -INFINITY, lsum = 0.f;
    // tr-read addresses of this lane inside a V image (block rows r0 + q, d columns of dt)
    const int grp = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    for (int ks = 0; ks < nst; ks++) {
        mm_wait_ahead<IPW, FA_NS>(min(FA_NS - 2, nst - 1 - ks));  // this wave's DMA of stage ks landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own ds_reads of the refilled stage retired
        __builtin_amdgcn_s_barrier();                              // ... every wave's; stage ks - 1 read
        asm volatile("" ::: "memory");
        if (ks + FA_NS - 1 < nst) issue((ks + FA_NS - 1) % FA_NS, ks + FA_NS - 1);
#pragma unroll
        for (int sub = 0; sub < FA_TPS; sub++) {
        const int b = 32 * ((st0 + ks) * FA_TPS + sub);
        if (b > last) break;  // wave-uniform: past this wave's rows (it still issues its DMA share)
        const char* kimg = fa_smem + (ks % FA_NS) * FA_STAGE_BYTES + sub * 2 * FA_TILE_BYTES;
        const char* vimg = kimg + FA_TILE_BYTES;
        // S^T = K Q^T
        f32x16 st = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            const f16x8 kf = *(const f16x8*)(kimg + fa_off(j32, 2 * ks + h));
            st = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qh[ks], st, 0, 0, 0);
            st = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, ql[ks], st, 0, 0, 0);
        }
        f16x8 ph[2], pl[2];
        fa_softmax_tile<NDT>(st, b, pos, h, inv_s * scale, b + 31 > pos0 + t0, m, lsum, o, ph, pl);
        // O^T += V^T P^T: element e of the A fragment = slot 16 s2 + 8 (e >> 2) + 4 h + (e & 3)
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++) {
#pragma unroll
            for (int dt = 0; dt < NDT; dt++) {
                const int r0 = 16 * s2 + 4 * h + qq, c0 = 4 * dt + 2 * (grp & 1) + (pp >> 1);
                typedef __attribute__((address_space(3))) fa_s16x4 lds_s16x4;
                const fa_s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(vimg + fa_off(r0, c0) + 8 * (pp & 1)));
                const fa_s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(vimg + fa_off(r0 + 8, c0) + 8 * (pp & 1)));
                typedef short s16x8 __attribute__((ext_vector_type(8)));
                const s16x8 xv = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
                const f16x8 vv = __builtin_bit_cast(f16x8, xv);
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vv, ph[s2], o[dt], 0, 0, 0);
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vv, pl[s2], o[dt], 0, 0, 0);
            }
        }
        }  // sub
    }
    const float l = lsum + __shfl_xor(lsum, 32);
    if (tq >= n) return;
    const bool split = nsplit > 1;
    const float inv_l = split ? 1.f : 1.f / l;
    float* orow = (split ? part_o + (size_t)z * n * q_stride : out) + (size_t)tq * q_stride + (size_t)head * HD;
    if (split && h == 0) part_ml[((size_t)z * n + tq) * (q_stride / HD) + head] = float2{m, l};
#pragma unroll
    for (int dt = 0; dt < NDT; dt++)
#pragma unroll
        for (int r = 0; r < 16; r += 4) {
            const int d = 32 * dt + 8 * (r >> 2) + 4 * h;
            *(float4*)(orow + d) =
                float4{o[dt][r] * inv_l, o[dt][r + 1] * inv_l, o[dt][r + 2] * inv_l, o[dt][r + 3] * inv_l};
        }
}

// the history splits of prefill_fa2_kernel combined per (token, head), in a fixed order:
// M = max m_z, out = sum_z e^(m_z - M) o_z / sum_z e^(m_z - M) l_z.  grid (n_heads, n), 256
// threads = 32 float4 columns of the head (HD = 128) x 8 split groups; group k takes splits
// k, k + 8, ... (its loads issued together), the 8 group sums are added in group order.
constexpr int FA_MERGE_GROUPS = 8;
__global__ __launch_bounds__(256) void prefill_fa_merge_kernel(const float* part_o, const float2* part_ml, float* out,
                                                               int n, int nsplit, int q_stride) {
    constexpr int G = FA_MERGE_GROUPS;
    __shared__ float smax[G];
    __shared__ float4 snum[G][32];
    __shared__ float sden[G];
    const int head = blockIdx.x, t = blockIdx.y;
    const int nh = gridDim.x;
    const int c = threadIdx.x & 31, k = threadIdx.x >> 5;
    auto ml_at = [&](const int z) { return part_ml[((size_t)z * n + t) * nh + head]; };
    float mx = -INFINITY;
    for (int z = k; z < nsplit; z += G) mx = fmaxf(mx, ml_at(z).x);
    if (c == 0) smax[k] = mx;
    __syncthreads();
    float M = smax[0];
#pragma unroll
    for (int i = 1; i < G; i++) M = fmaxf(M, smax[i]);
    float4 acc = float4{0.f, 0.f, 0.f, 0.f};
    float l = 0.f;
    for (int z = k; z < nsplit; z += G) {
        const float2 m_l = ml_at(z);
        const float w = __expf(m_l.x - M);
        const float4 v = *(const float4*)(part_o + ((size_t)z * n + t) * q_stride + (size_t)head * 128 + 4 * c);
        l += w * m_l.y;
        acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
    }
    snum[k][c] = acc;
    if (c == 0) sden[k] = l;
    __syncthreads();
    if (k == 0) {
        float4 s4 = snum[0][c];
        float den = sden[0];
#pragma unroll
        for (int i = 1; i < G; i++) {
            s4.x += snum[i][c].x; s4.y += snum[i][c].y; s4.z += snum[i][c].z; s4.w += snum[i][c].w;
            den += sden[i];
        }
        const float inv_l = 1.f / den;
        *(float4*)(out + (size_t)t * q_stride + (size_t)head * 128 + 4 * c) =
            float4{s4.x * inv_l, s4.y * inv_l, s4.z * inv_l, s4.w * inv_l};
    }
}

// fp8 weights (e4m3 / e5m2, finite codes only: the _EXACT dtypes never come here) -> f16 bits
// for the hipBLASLt f16 GEMM of a prompt pass.  Every finite e4m3 / e5m2 value is an f16, so
// the GEMM multiplies exactly the reference's decoded weights (src/types.h:302-314); the
// pack's round-toward-zero never rounds.  n16: 16-byte chunks of codes; out: 2 n16 chunks.
template <int DT>
__global__ __launch_bounds__(256) void pf_dequant_f16_kernel(const u32x4* w, const size_t n16, u32x4* out) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const u32x4 v = __builtin_nontemporal_load(w + i);
        float f[16];
        WDec<DT>::dec(v, f);
        uint32_t h[8];
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(f[2 * j], f[2 * j + 1]));
        out[2 * i] = u32x4{h[0], h[1], h[2], h[3]};
        out[2 * i + 1] = u32x4{h[4], h[5], h[6], h[7]};
    }
}

// gguf blocks (Q8_0 / Q4_0, planar device rows: codes, then one f16 scale d per 32 elements) ->
// the exact f16 hi + lo of every weight for the f16 GEMMs of a prompt pass.  The converter's
// value d * q (quants.py: Q8_0 :448-454, Q4_0 :302-311) is exact in f32 (11-bit d times a 4- or
// 8-bit q) and splits exactly into hi = f16(v) and lo = f16(v - hi) (at most 19 significant bits,
// and lo a multiple of d's ulp), so W = W_hi + W_lo with no rounding: the GEMM runs once over
// each image.  One thread per 8 consecutive elements of a row; hi / lo: [rows][K].
template <int DT>
__global__ __launch_bounds__(256) void pf_dequant_gq_kernel(const uint8_t* w, const int rows, const int K,
                                                           uint16_t* hi, uint16_t* lo) {
    const size_t pitch = gq_pitch(DT, (size_t)K), qbytes = gq_qbytes(DT, (size_t)K);
    const size_t per_row = (size_t)K / 8, total = (size_t)rows * per_row;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        const size_t r = i / per_row;
        const int k = (int)(i - r * per_row) * 8;  // 8 elements k .. k+7 of one block
        const uint8_t* row = w + r * pitch;
        const int b = k >> 5, j0 = k & 31;
        const float d = f16_bits_to_f32(*(const uint16_t*)(row + qbytes + 2 * b));
        int q[8];
        if constexpr (DT == XH_Q8_0) {
            const uint2 u = *(const uint2*)(row + k);
#pragma unroll
            for (int e = 0; e < 8; e++) q[e] = (int8_t)(((e < 4 ? u.x : u.y) >> (8 * (e & 3))) & 0xffu);
        } else {
            // element j of a block: byte j & 15 of its 16, low nibble for j < 16, high for j >= 16
            const uint2 u = *(const uint2*)(row + 16 * b + (j0 & 15));
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const uint32_t byte = ((e < 4 ? u.x : u.y) >> (8 * (e & 3))) & 0xffu;
                q[e] = (int)(j0 < 16 ? (byte & 15u) : (byte >> 4)) - 8;
            }
        }
        uint32_t h[4], l[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            const float v0 = d * (float)q[e], v1 = d * (float)q[e + 1];
            const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
            const _Float16 l0 = (_Float16)(v0 - (float)h0), l1 = (_Float16)(v1 - (float)h1);
            h[e / 2] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
            l[e / 2] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
        }
        *(u32x4*)(hi + r * (size_t)K + k) = u32x4{h[0], h[1], h[2], h[3]};
        *(u32x4*)(lo + r * (size_t)K + k) = u32x4{l[0], l[1], l[2], l[3]};
    }
}

}  // namespace xalm
