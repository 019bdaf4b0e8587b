// gemv.h — batch-1 weight-streaming matvec for gfx950 with fused prologues/epilogues.
//
// Replaces `matmul<TX,TW>` (jubruckne/Xalm src/infer.cpp:104-135, dispatch :185-216) and
// the elementwise ops around each call site in Block::_block_cpu (src/infer.cpp:365-496):
//   prologue  PRO_RMSNORM : rmsnorm(xb, x, w) (src/infer.cpp:224-236) recomputed per block
//   epilogue  EPI_QKV     : qkv clip (:392-399), rope (:305-322, :407-408), fp16 KV write (:410-414)
//             EPI_GLU     : hb = act(W1 x) * (W3 x) (:468-488), W1/W3 rows interleaved
//             EPI_RESID   : x += W x (:447-452, :490-494)
//             EPI_STORE   : y = W x (logits, :637)
//             EPI_LOGITS  : EPI_STORE + one argmax candidate per workgroup (Sampler::sample_argmax,
//                           src/sampler.cpp:19-30), for the device decode loop
//
// HBM layout: W row-major [rows][n] exactly as the .xalm tensor (HF [out,in]).  One wave
// owns ROWS consecutive rows; lane l streams 16-byte chunks l, l+64, l+128, ... of each row
// (1 KiB per wave-instruction per row, fully coalesced), U chunks per row in flight, with
// non-temporal loads (weights are read once per token).  The activation vector is staged once
// per workgroup in LDS in a lane-permuted layout so every lane reads its x values with
// conflict-free ds_read_b128.  Dot products reduce across the wave with cross-lane shuffles;
// no MFMA: batch-1 matvec is HBM-bound at ~1 FLOP per weight byte.
#pragma once

#include <float.h>

#include "common.h"

namespace xalm {

enum { PRO_PLAIN = 0, PRO_RMSNORM = 1 };
enum { EPI_STORE = 0, EPI_RESID = 1, EPI_QKV = 2, EPI_GLU = 3, EPI_LOGITS = 4 };

constexpr int LDS_HEAD_BYTES = 64;
#ifndef GEMV_BAL_CU
#define GEMV_BAL_CU 256
#endif  // block-reduction scratch in front of the x image

// attn_wo.h hand-off words of a layer that the launch after it zeroes (every 32nd word)
constexpr int AW_RESET_WORDS = 9;

// Launch shape of one gemv instance.
template <int THREADS_, int ROWS_, int U_, bool NT_ = true, int MINW_ = 4, bool PF_ = true, int XN_ = 0, int PIPE_ = 1,
          bool BAL_ = false>
struct GemvShape {
    static constexpr bool BAL = BAL_;          // grid in whole multiples of the CU count, groups
                                               // in wave-major order (gemv_blocks, gemv_body)
    static constexpr int PIPE = PIPE_;         // 2: two register sets (gemv_rows_pipe; host-checked
                                               // n % (64 E U) == 0, no gguf blocks)
    static constexpr int THREADS = THREADS_;   // workgroup size
    static constexpr int WAVES = THREADS_ / 64;
    static constexpr int ROWS = ROWS_;         // rows per wave and group (even for QKV / GLU)
    static constexpr int U = U_;               // 16-B chunks per row in flight
    static constexpr bool NT = NT_;            // non-temporal weight loads
    static constexpr int MINW = MINW_;         // __launch_bounds__ min waves per SIMD
    static constexpr bool PF = PF_;            // first U chunks requested inside the x prologue
    static constexpr int XN = XN_;             // PF: float4 of x (and norm) per thread held in registers
};

struct GemvArgs {
    const void* w;        // [rows][n]
    size_t row_bytes;     // n * sizeof(element)
    int n;                // input length
    int rows;             // output rows
    const float* x;       // input [n], fp32
    const void* norm_w;   // PRO_RMSNORM weight [n] (F32 or BF16)
    int norm_dtype;
    float eps;
    float* out;           // EPI_STORE / EPI_RESID: [rows];  EPI_GLU: [rows/2]
    // EPI_QKV
    float* q;             // [q_dim]
    uint16_t* kcache;     // this layer's K ring [max_seq_len][kv_dim] (fp16 bits)
    uint16_t* vcache;
    int q_dim;
    int kv_dim;
    int head_dim;
    const float* rope_freq;  // [head_dim/2]: 1/powf(theta, j/rotary_dim) or 0 (host libm)
    const float* rope_cs;    // [head_dim]: cosf, then sinf of (float)pos * rope_freq[j] at this step's
                             // pos (rope_table, computed once per step by its embed kernel)
    const float* sink_cos;   // [head_dim/2]: cosf(freq) (rope at pos=1, host libm)
    const float* sink_sin;
    float qkv_clip;
    int act;
    const StepParams* sp;
    unsigned long long* trace;  // debug (null = off): per workgroup [4] start, x staged, rows done
    unsigned long long* cand;   // EPI_LOGITS: [gridDim.x] argmax_key of the workgroup's best logit
    unsigned* aw_reset;         // workgroup 0 zeroes words 0, 32, ..., 32 (AW_RESET_WORDS - 1) (attn_wo.h sync)
};

// agent-scope relaxed (sc1: L1-bypassing, write-through) accesses for data handed between
// workgroups of one launch
__device__ __forceinline__ uint32_t ld_sc1_u32(const void* p) {
    return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_u32(void* p, const uint32_t v) {
    __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1_f(const float* p) { return __builtin_bit_cast(float, ld_sc1_u32(p)); }
__device__ __forceinline__ void st_sc1_f(float* p, const float v) { st_sc1_u32(p, __builtin_bit_cast(uint32_t, v)); }

__device__ __forceinline__ float clipf(const float x, const float v) { return x < -v ? -v : (x > v ? v : x); }


// One rope rotation of the adjacent pair (v0, v1) at frequency freq (src/infer.cpp:308-321).
__device__ __forceinline__ void rope_pair_f(float& v0, float& v1, const float freq, const int pos) {
    const float val = (float)pos * freq;
    const float fcr = cosf(val);
    const float fci = sinf(val);
    const float a = v0, b = v1;
    v0 = a * fcr - b * fci;
    v1 = a * fci + b * fcr;
}
// ... at element index i (frequency from the table)
__device__ __forceinline__ void rope_pair(float& v0, float& v1, const int i, const int head_dim, const int pos,
                                          const float* freq_tab) {
    const int j_head = i % head_dim;
    const float freq = freq_tab[j_head >> 1];
    const float val = (float)pos * freq;
    const float fcr = cosf(val);
    const float fci = sinf(val);
    const float a = v0, b = v1;
    v0 = a * fcr - b * fci;
    v1 = a * fci + b * fcr;
}

// ... with the rotation's cosf / sinf given (the values rope_pair_f computes: rope_table below)
__device__ __forceinline__ void rope_pair_cs(float& v0, float& v1, const float fcr, const float fci) {
    const float a = v0, b = v1;
    v0 = a * fcr - b * fci;
    v1 = a * fci + b * fcr;
}
// ... at element index i from the step's table [cos | sin]
__device__ __forceinline__ void rope_pair_tab(float& v0, float& v1, const int i, const int head_dim, const float* cs) {
    const int j = (i % head_dim) >> 1;
    rope_pair_cs(v0, v1, cs[j], cs[(head_dim >> 1) + j]);
}
// the step's rotations, by threads j < head_dim / 2 of one workgroup: cs[j] = cosf(pos * freq[j]),
// cs[head_dim / 2 + j] = sinf(...) (rope_pair's arithmetic, src/infer.cpp:308-321, once per step
// instead of once per row pair in every qkv epilogue)
__device__ __forceinline__ void rope_table(float* cs, const float* freq, const int half, const int pos, const int j) {
    if (j < half) {
        const float val = (float)pos * freq[j];
        cs[j] = cosf(val);
        cs[half + j] = sinf(val);
    }
}

// Sum of squares of x[0..n) -> rms scale 1/sqrtf(ss/n + eps), identical in every block of one
// launch (fixed per-thread stride order, fixed shuffle tree, fixed wave order).
template <int THREADS>
__device__ __forceinline__ float block_rms_scale(const float* x, const int n, const float eps, float* red) {
    const int tid = threadIdx.x;
    const float4* x4 = (const float4*)x;
    float ss = 0.f;
    for (int i = tid; i < (n >> 2); i += THREADS) {
        const float4 v = x4[i];
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = wave_sum(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < THREADS / 64; w++) tot += red[w];
    const float rms = sqrtf(tot / (float)n + eps);
    return 1.0f / rms;
}

__device__ __forceinline__ float4 load_norm4(const void* w, const int dtype, const int i4) {
    if (dtype == XH_BF16) {
        const uint2 u = ((const uint2*)w)[i4];
        return make_float4(bits_f32(u.x << 16), bits_f32(u.x & 0xffff0000u), bits_f32(u.y << 16),
                           bits_f32(u.y & 0xffff0000u));
    }
    return ((const float4*)w)[i4];
}

// Branch-free form of load_norm4 for the PF prologue: one 16-byte buffer load at the
// dtype's stride (bounds-checked by the descriptor: the bytes past the vector read as 0), then
// selects.  norm dtype is F32 or BF16.
__device__ __forceinline__ float4 load_norm4_nb(const void* w, const int dtype, const int n, const int i4) {
    const bool bf = dtype == XH_BF16;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, n * (bf ? 2 : 4), 0x00020000);
    const u32x4 u = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, i4 * (bf ? 8 : 16), 0, 0));
    return make_float4(bf ? bits_f32(u.x << 16) : bits_f32(u.x), bf ? bits_f32(u.x & 0xffff0000u) : bits_f32(u.y),
                       bf ? bits_f32(u.y << 16) : bits_f32(u.z), bf ? bits_f32(u.y & 0xffff0000u) : bits_f32(u.w));
}

// Q4_0 staging (the denormal form of gq_dot): the image holds x / 16 for elements 16..31 of each
// 32-element block and, after the n_it * 64 * E floats of the image, -8 sum(x) of every block
template <int DT>
__device__ __host__ constexpr bool gq4_image() { return DT == XH_Q4_0; }
__device__ __forceinline__ const float* gq4_nxs(const float4* xs4, const int n) {
    constexpr int E = 32;
    return (const float*)xs4 + (size_t)((n + 64 * E - 1) / (64 * E)) * 64 * E;
}
// one float4 v = x[4 i .. 4 i + 3] into the image slot of a Q4_0 block (lanes 8 k .. 8 k + 7 hold
// the 8 float4 of block k, i % 8 == lane % 8): the sum over the block in a fixed shuffle tree, the
// block's -8 sum(x) stored by its first lane; valid: i < n / 4 (the 8 lanes agree)
__device__ __forceinline__ float4 gq4_stage(float4 v, const int i, const bool valid, float4* xs4, const int n) {
    const float t = group_reduce<8>((v.x + v.y) + (v.z + v.w));  // DPP: no LDS round trips
    if (valid && (i & 7) == 0) ((float*)gq4_nxs(xs4, n))[i >> 3] = -8.f * t;
    const float f = (i & 4) ? 0.0625f : 1.f;  // elements 16..31 of the block: x / 16 (exact)
    v.x *= f; v.y *= f; v.z *= f; v.w *= f;
    return v;
}

// x (optionally rms-normalised and weighted) -> LDS image xs4, permuted so that lane l at
// chunk `it` finds the E/4 float4 it multiplies at xs4[(it*E/4 + q)*64 + l].
// SC1: x was published inside the running launch (write-through): read it with sc1 loads.
template <int E, int PRO, int THREADS, bool SC1 = false, bool GQ4 = false>
__device__ __forceinline__ void stage_x(const GemvArgs& a, float4* xs4, float* red) {
    const int n = a.n;
    float scale = 1.f;
    if (PRO == PRO_RMSNORM) scale = block_rms_scale<THREADS>(a.x, n, a.eps, red);
    const float4* x4 = (const float4*)a.x;
    for (int i = threadIdx.x; i < (n >> 2); i += THREADS) {
        float4 v;
        if (SC1) {
            const u32x4 u = ld_sc1_x4(a.x, (uint32_t)i * 16);
            v = make_float4(bits_f32(u.x), bits_f32(u.y), bits_f32(u.z), bits_f32(u.w));
        } else {
            v = x4[i];
        }
        if (PRO == PRO_RMSNORM) {
            const float4 w = load_norm4(a.norm_w, a.norm_dtype, i);
            v.x = v.x * scale * w.x;  // x[i] * scale * weight[i], src/infer.cpp:234
            v.y = v.y * scale * w.y;
            v.z = v.z * scale * w.z;
            v.w = v.w * scale * w.w;
        }
        if constexpr (GQ4) v = gq4_stage(v, i, true, xs4, n);
        const int c = i << 2;
        const int it = c / (64 * E);
        const int rem = c - it * 64 * E;
        const int l = rem / E;
        const int qd = (rem - l * E) >> 2;
        xs4[(it * (E / 4) + qd) * 64 + l] = v;
    }
}

// StreamingLLM sink re-rotation (src/infer.cpp:421-431): K[r] = f16(rope(f32(K[r]), pos=1)).
template <int THREADS>
__device__ __forceinline__ void rotate_sinks(const GemvArgs& a, const int kv_sink) {
    for (int r = 0; r < kv_sink; r++) {
        uint16_t* krow = a.kcache + (size_t)r * a.kv_dim;
        for (int p = threadIdx.x; p < (a.kv_dim >> 1); p += THREADS) {
            const int i = p << 1;
            const int jh = (i % a.head_dim) >> 1;
            const float k0 = f16_bits_to_f32(krow[i]), k1 = f16_bits_to_f32(krow[i + 1]);
            const float fcr = a.sink_cos[jh], fci = a.sink_sin[jh];
            krow[i] = f32_to_f16_bits(k0 * fcr - k1 * fci);
            krow[i + 1] = f32_to_f16_bits(k0 * fci + k1 * fcr);
        }
    }
}

// SC1: activations another workgroup of the same launch reads are stored write-through, and
// the residual it may have written is read with sc1 loads; otherwise plain accesses.
template <bool SC1>
__device__ __forceinline__ void epi_st(float* p, const float v) {
    if (SC1) st_sc1_f(p, v);
    else *p = v;
}
// QKV epilogue inputs requested ahead of the group's weights (gemv_rows_pipe): the step's
// position, ring slot and the rope frequency of each row pair, so the epilogue at the group's
// end does not start two dependent loads (StepParams, then the frequency table)
template <int ROWS>
struct QkvPre {
    int pos, kv_pos;
    float cs[ROWS >= 2 ? ROWS : 2];  // (cos, sin) of each row pair's rotation
};
// res: EPI_RESID's residual rows, requested with the group's first weights (not from the
// epilogue, where the load would be a dependent round trip at the group's end)
template <int EPI, int ROWS, bool SC1 = false>
__device__ __forceinline__ void gemv_epilogue(const GemvArgs& a, const int row0, const float* acc,
                                              unsigned long long* best = nullptr,
                                              const QkvPre<ROWS>* pre = nullptr, const float* res = nullptr) {
    if (EPI == EPI_LOGITS) {
#pragma unroll
        for (int r = 0; r < ROWS; r++)
            if (row0 + r < a.rows) {
                a.out[row0 + r] = acc[r];
                // only logits > FLT_MIN compete (max_val starts at FLT_MIN, strict '>')
                if (acc[r] > FLT_MIN) {
                    const unsigned long long k = argmax_key(acc[r], row0 + r);
                    *best = k > *best ? k : *best;
                }
            }
    } else if (EPI == EPI_STORE) {
#pragma unroll
        for (int r = 0; r < ROWS; r++)
            if (row0 + r < a.rows) epi_st<SC1>(a.out + row0 + r, acc[r]);
    } else if (EPI == EPI_RESID) {
#pragma unroll
        for (int r = 0; r < ROWS; r++)
            if (row0 + r < a.rows)
                epi_st<SC1>(a.out + row0 + r, (res ? res[r] : SC1 ? ld_sc1_f(a.out + row0 + r) : a.out[row0 + r]) + acc[r]);
    } else if (EPI == EPI_GLU) {
#pragma unroll
        for (int p = 0; p < ROWS; p += 2) epi_st<SC1>(a.out + ((row0 + p) >> 1), act_fn(a.act, acc[p]) * acc[p + 1]);
    } else {  // EPI_QKV
        const int kv_pos = pre ? pre->kv_pos : a.sp->kv_pos;
#pragma unroll
        for (int p = 0; p < ROWS; p += 2) {
            const int row = row0 + p;
            float v0 = clipf(acc[p], a.qkv_clip), v1 = clipf(acc[p + 1], a.qkv_clip);
            if (row < a.q_dim) {
                if (pre) rope_pair_cs(v0, v1, pre->cs[p], pre->cs[p + 1]);
                else rope_pair_tab(v0, v1, row, a.head_dim, a.rope_cs);
                epi_st<SC1>(a.q + row, v0);
                epi_st<SC1>(a.q + row + 1, v1);
            } else {
                const bool isk = row < a.q_dim + a.kv_dim;
                const int kr = isk ? row - a.q_dim : row - a.q_dim - a.kv_dim;
                if (isk) {
                    if (pre) rope_pair_cs(v0, v1, pre->cs[p], pre->cs[p + 1]);  // q_dim % head_dim == 0
                    else rope_pair_tab(v0, v1, kr, a.head_dim, a.rope_cs);
                }
                uint16_t* dst = (isk ? a.kcache : a.vcache) + (size_t)kv_pos * a.kv_dim + kr;
                // the pair as one 4-byte store (kr is even)
                const uint32_t pk = (uint32_t)f32_to_f16_bits(v0) | ((uint32_t)f32_to_f16_bits(v1) << 16);
                if (SC1) st_sc1_u32(dst, pk);
                else *(uint32_t*)dst = pk;
            }
        }
    }
}

// Weight chunks [it, it+U) of a row group: U x ROWS 16-byte loads per lane, straight to VGPRs.
template <int ROWS, int U, bool NT>
__device__ __forceinline__ void gemv_load(u32x4 (&wv)[U][ROWS], const char* wrow, const size_t row_bytes,
                                          const int it) {
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            // global address space: stays a global_load even where the pointer's origin is opaque
            const __attribute__((address_space(1))) u32x4* p =
                (const __attribute__((address_space(1))) u32x4*)(wrow + (size_t)r * row_bytes + (size_t)(it + u) * 1024);
            wv[u][r] = NT ? __builtin_nontemporal_load(p) : *p;
        }
}

__device__ __forceinline__ float fma_mix_lo(const uint32_t h2, const float x, float acc);
__device__ __forceinline__ float fma_mix_hi(const uint32_t h2, const float x, float acc);

template <int DT, int ROWS, int U>
__device__ __forceinline__ void gemv_compute(const u32x4 (&wv)[U][ROWS], const float4* xs4, const int it,
                                             const int lane, float* acc) {
    constexpr int E = WDec<DT>::E;
    constexpr int QN = E / 4;
#pragma unroll
    for (int u = 0; u < U; u++) {
        float4 xv[QN];
#pragma unroll
        for (int qd = 0; qd < QN; qd++) xv[qd] = xs4[((it + u) * QN + qd) * 64 + lane];
        if constexpr (DT == XH_F16) {
            // f16 weights: v_fma_mix_f32 takes the f16 half directly (one op per element instead
            // of a convert and an fma; the convert is exact, so the sums are bit-identical)
#pragma unroll
            for (int r = 0; r < ROWS; r++) {
                float s = acc[r];
                const uint32_t w4[4] = {wv[u][r].x, wv[u][r].y, wv[u][r].z, wv[u][r].w};
#pragma unroll
                for (int qd = 0; qd < QN; qd++) {
                    s = fma_mix_lo(w4[2 * qd], xv[qd].x, s);
                    s = fma_mix_hi(w4[2 * qd], xv[qd].y, s);
                    s = fma_mix_lo(w4[2 * qd + 1], xv[qd].z, s);
                    s = fma_mix_hi(w4[2 * qd + 1], xv[qd].w, s);
                }
                acc[r] = s;
            }
            continue;
        }
        if constexpr (DT == XH_F8_E4M3 || DT == XH_F8_E5M2) {
            // fp8 pairs straight from v_cvt_pk_f32_fp8 / _bf8 into v_pk_fma_f32 (even and odd
            // elements of the chunk in the two halves, added at the chunk's end): 598 -> 605 tok/s
            // fp8 Mistral-7B decode (same-box A/B, two rounds)
#pragma unroll
            for (int r = 0; r < ROWS; r++) {
                const uint32_t w4[4] = {wv[u][r].x, wv[u][r].y, wv[u][r].z, wv[u][r].w};
                f2_t s2 = {acc[r], 0.f};
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const f2_t lo = DT == XH_F8_E5M2 ? __builtin_amdgcn_cvt_pk_f32_bf8(w4[i], false)
                                                     : __builtin_amdgcn_cvt_pk_f32_fp8(w4[i], false);
                    const f2_t hi = DT == XH_F8_E5M2 ? __builtin_amdgcn_cvt_pk_f32_bf8(w4[i], true)
                                                     : __builtin_amdgcn_cvt_pk_f32_fp8(w4[i], true);
                    s2 = __builtin_elementwise_fma(lo, f2_t{xv[i].x, xv[i].y}, s2);
                    s2 = __builtin_elementwise_fma(hi, f2_t{xv[i].z, xv[i].w}, s2);
                }
                acc[r] = s2.x + s2.y;
            }
            continue;
        }
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            float f[E];
            WDec<DT>::dec(wv[u][r], f);
            float s = acc[r];
#pragma unroll
            for (int qd = 0; qd < QN; qd++) {
                s = fmaf(f[4 * qd + 0], xv[qd].x, s);
                s = fmaf(f[4 * qd + 1], xv[qd].y, s);
                s = fmaf(f[4 * qd + 2], xv[qd].z, s);
                s = fmaf(f[4 * qd + 3], xv[qd].w, s);
            }
            acc[r] = s;
        }
    }
}

template <int DT, int ROWS, int U, bool NT>
__device__ __forceinline__ void gemv_chunk(const char* wrow, const size_t row_bytes, const float4* xs4, const int it,
                                           const int lane, float* acc) {
    u32x4 wv[U][ROWS];
    gemv_load<ROWS, U, NT>(wv, wrow, row_bytes, it);
    gemv_compute<DT, ROWS, U>(wv, xs4, it, lane, acc);
}

// sum of q * x over one 16-B chunk of gguf codes against the chunk's x floats (xv: E/4 float4).
// The codes become exact packed f16 with the magic-number form (byte b placed under the f16
// exponent of 1024 by v_perm_b32: 1024 + b, then one packed subtract of 1024 + bias), and
// v_fma_mix_f32 multiplies an f16 half by the f32 x and accumulates in f32: 2.25 (Q8_0) /
// 2.4 (Q4_0) VALU ops per element instead of an integer extract, convert and fma each.
__device__ __forceinline__ float fma_mix_lo(const uint32_t h2, const float x, float acc) {
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(h2), "v"(x));
    return acc;
}
__device__ __forceinline__ float fma_mix_hi(const uint32_t h2, const float x, float acc) {
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(h2), "v"(x));
    return acc;
}
// bytes 0 and 1 (sel 0x04010400) or 2 and 3 (0x04030402) of b as two f16 1024 + byte, minus c
__device__ __forceinline__ uint32_t gq_pair(const uint32_t b, const uint32_t sel, const h2_t c) {
    const uint32_t p = __builtin_amdgcn_perm(0x64646464u, b, sel);
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(h2_t, p) + c);
}
template <int DT>
__device__ __forceinline__ float gq_dot(const u32x4 w, const float4* xv) {
    const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
    float s = 0.f;
    if constexpr (DT == XH_Q8_0) {
        // int8 q: b = q + 128 (xor 0x80), 1024 + b - 1152 = q
        const h2_t c = __builtin_bit_cast(h2_t, 0xE480E480u);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t u = ww[i] ^ 0x80808080u;
            const uint32_t p01 = gq_pair(u, 0x04010400u, c), p23 = gq_pair(u, 0x04030402u, c);
            s = fma_mix_lo(p01, xv[i].x, s);
            s = fma_mix_hi(p01, xv[i].y, s);
            s = fma_mix_lo(p23, xv[i].z, s);
            s = fma_mix_hi(p23, xv[i].w, s);
        }
    } else {
        // Q4_0 (byte j = element j in the low nibble, j + 16 in the high one), denormal form: the
        // nibbles are masked into the mantissa bits of packed f16 with a zero exponent, so each
        // f16 reads n * 2^-24 exactly (low nibbles of bytes 0 / 2, and of bytes 1 / 3 after >> 8)
        // or 16 n * 2^-24 (high nibbles in place, against the image's x / 16 for elements 16..31,
        // exact): 13 VALU ops per 8 elements instead of 19.  The result is sum(n x) * 2^-24; the
        // caller forms sum((n - 8) x) = 2^24 * s - 8 * sum(x) with the block's staged -8 sum(x).
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t w8 = ww[i] >> 8;
            const uint32_t a = ww[i] & 0x000F000Fu, b = w8 & 0x000F000Fu;
            const uint32_t c = ww[i] & 0x00F000F0u, d = w8 & 0x00F000F0u;
            s = fma_mix_lo(a, xv[i].x, s);
            s = fma_mix_lo(b, xv[i].y, s);
            s = fma_mix_hi(a, xv[i].z, s);
            s = fma_mix_hi(b, xv[i].w, s);
            s = fma_mix_lo(c, xv[4 + i].x, s);
            s = fma_mix_lo(d, xv[4 + i].y, s);
            s = fma_mix_hi(c, xv[4 + i].z, s);
            s = fma_mix_hi(d, xv[4 + i].w, s);
        }
    }
    return s;
}

// acc[r] += d[r] * sum(q * x) for the ROWS rows of one chunk (Q4_0: nx = -8 sum(x) of the block)
template <int DT, int ROWS>
__device__ __forceinline__ void gq_rows(const u32x4 (&w)[ROWS], const float (&d)[ROWS], const float4* xv, float* acc,
                                        const float nx) {
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        if constexpr (DT == XH_Q4_0) acc[r] = fmaf(d[r], fmaf(gq_dot<DT>(w[r], xv), 0x1p24f, nx), acc[r]);
        else acc[r] = fmaf(d[r], gq_dot<DT>(w[r], xv), acc[r]);
    }
}

// gguf blocks (WScale<DT>::BLOCK = 32): chunks [it, it+U) as gemv_chunk, and each chunk's f16
// block scale d from the planar row tail (qbytes = quant bytes per row); a chunk's partial dot
// product is scaled once: acc += d * sum(q * x)  (quants.py dequantizes d*q per element; the
// same sum up to f32 reassociation)
template <int DT, int ROWS, int U, bool NT>
__device__ __forceinline__ void gemv_chunk_gq(const char* wrow, const size_t row_bytes, const size_t qbytes,
                                              const float4* xs4, const int it, const int lane, float* acc,
                                              const float* nxs) {
    constexpr int E = WDec<DT>::E;
    constexpr int QN = E / 4;
    u32x4 wv[U][ROWS];
    gemv_load<ROWS, U, NT>(wv, wrow, row_bytes, it);
    float d[U][ROWS];
    const char* rb = wrow - lane * 16 + qbytes;
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const int blk = (((it + u) * 64 + lane) * E) / WScale<DT>::BLOCK;
            d[u][r] = (float)__builtin_bit_cast(_Float16, *(const uint16_t*)(rb + (size_t)r * row_bytes + blk * 2));
        }
#pragma unroll
    for (int u = 0; u < U; u++) {
        float4 xv[QN];
#pragma unroll
        for (int qd = 0; qd < QN; qd++) xv[qd] = xs4[((it + u) * QN + qd) * 64 + lane];
        gq_rows<DT, ROWS>(wv[u], d[u], xv, acc, gq4_image<DT>() ? nxs[(it + u) * 64 + lane] : 0.f);
    }
}

// gguf blocks, split in two for the pipelined stream: the f16 block scale d of each of the
// chunks [it, it+U) of a row group (wrow: this lane's pointer into the group's first row)...
template <int DT, int ROWS, int U>
__device__ __forceinline__ void gq_load_scales(float (&d)[U][ROWS], const char* wrow, const size_t row_bytes,
                                               const size_t qbytes, const int it, const int lane) {
    constexpr int E = WDec<DT>::E;
    const char* rb = wrow - lane * 16 + qbytes;
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const int blk = (((it + u) * 64 + lane) * E) / WScale<DT>::BLOCK;
            d[u][r] = (float)__builtin_bit_cast(_Float16, *(const uint16_t*)(rb + (size_t)r * row_bytes + blk * 2));
        }
}
// ...and the scaled chunk sums against the staged x, as gemv_chunk_gq
template <int DT, int ROWS, int U>
__device__ __forceinline__ void gq_compute(const u32x4 (&wv)[U][ROWS], const float (&d)[U][ROWS], const float4* xs4,
                                           const int it, const int lane, float* acc, const float* nxs) {
    constexpr int QN = WDec<DT>::E / 4;
#pragma unroll
    for (int u = 0; u < U; u++) {
        float4 xv[QN];
#pragma unroll
        for (int qd = 0; qd < QN; qd++) xv[qd] = xs4[((it + u) * QN + qd) * 64 + lane];
        gq_rows<DT, ROWS>(wv[u], d[u], xv, acc, gq4_image<DT>() ? nxs[(it + u) * 64 + lane] : 0.f);
    }
}

// Row group `grp` of the matrix: lane pointer and row stride (0 for the duplicated last row
// of an odd row count: rows past the end re-read the last row and are never stored).
template <int ROWS>
__device__ __forceinline__ const char* gemv_row_ptr(const GemvArgs& a, const int grp, const int lane, size_t& rstride) {
    const int rmax = a.rows - 1;
    const int row0 = grp * ROWS;
    rstride = (row0 + ROWS - 1 <= rmax) ? a.row_bytes : 0;
    return (const char*)a.w + (size_t)(row0 < rmax ? row0 : rmax) * a.row_bytes + lane * 16;
}
template <class S>
__device__ __forceinline__ int gemv_groups(const GemvArgs& a) { return (a.rows + S::ROWS - 1) / S::ROWS; }

// chunks [0, U) of group g into pre (the caller checked g < groups and n_full >= U)
template <class S>
__device__ __forceinline__ void gemv_prefetch(const GemvArgs& a, const int g, const int lane,
                                              u32x4 (&pre)[S::U][S::ROWS]) {
    size_t rs;
    const char* wrow = gemv_row_ptr<S::ROWS>(a, g, lane, rs);
    gemv_load<S::ROWS, S::U, S::NT>(pre, wrow, rs, 0);
}

// Chunks [it, n) of group g into acc, then the wave reduction and the epilogue.
template <int DT, int EPI, class S, bool SC1 = false>
__device__ __forceinline__ void gemv_group(const GemvArgs& a, const int g, const int lane, const float4* xs4, float* acc,
                                           int it, unsigned long long* best = nullptr) {
    constexpr int ROWS = S::ROWS, U = S::U;
    constexpr int E = WDec<DT>::E;
    const int n = a.n;
    const int n_full = n / (64 * E);
    const int n_it = (n + 64 * E - 1) / (64 * E);
    size_t rstride;
    const char* wrow = gemv_row_ptr<ROWS>(a, g, lane, rstride);
    constexpr bool RES = EPI == EPI_RESID && !SC1;
    float res[ROWS];
    if constexpr (RES) {
#pragma unroll
        for (int r = 0; r < ROWS; r++) res[r] = a.out[min(g * ROWS + r, a.rows - 1)];
    }
    if constexpr (WScale<DT>::BLOCK > 0) {
        const size_t qb = gq_qbytes(DT, (size_t)n);
        const float* nxs = gq4_image<DT>() ? gq4_nxs(xs4, n) : nullptr;
        for (; it + U <= n_full; it += U) gemv_chunk_gq<DT, ROWS, U, S::NT>(wrow, rstride, qb, xs4, it, lane, acc, nxs);
        if (U > 2)
            for (; it + 2 <= n_full; it += 2)
                gemv_chunk_gq<DT, ROWS, 2, S::NT>(wrow, rstride, qb, xs4, it, lane, acc, nxs);
        for (; it < n_full; it++) gemv_chunk_gq<DT, ROWS, 1, S::NT>(wrow, rstride, qb, xs4, it, lane, acc, nxs);
        if (it < n_it && (it * 64 + lane) * E < n)
            gemv_chunk_gq<DT, ROWS, 1, S::NT>(wrow, rstride, qb, xs4, it, lane, acc, nxs);
    } else {
        for (; it + U <= n_full; it += U) gemv_chunk<DT, ROWS, U, S::NT>(wrow, rstride, xs4, it, lane, acc);
        if (U > 2)
            for (; it + 2 <= n_full; it += 2) gemv_chunk<DT, ROWS, 2, S::NT>(wrow, rstride, xs4, it, lane, acc);
        for (; it < n_full; it++) gemv_chunk<DT, ROWS, 1, S::NT>(wrow, rstride, xs4, it, lane, acc);
        if (it < n_it && (it * 64 + lane) * E < n) gemv_chunk<DT, ROWS, 1, S::NT>(wrow, rstride, xs4, it, lane, acc);
    }
#pragma unroll
    for (int r = 0; r < ROWS; r++) acc[r] = wave_sum(acc[r]);
    if (lane == 0) gemv_epilogue<EPI, ROWS, SC1>(a, g * ROWS, acc, best, nullptr, RES ? res : nullptr);
}

// Groups g, g + total_waves, ... of this wave against the staged x image.  FIRST: the first
// group's chunks [0, U) are already in `pre` (the caller checked g < groups and n_full >= U);
// that group is peeled so `pre` is dead in the loop.
template <int DT, int EPI, class S, bool FIRST, bool SC1 = false>
__device__ __forceinline__ void gemv_rows(const GemvArgs& a, int g, const int total_waves, const int lane,
                                          const float4* xs4, const u32x4 (&pre)[S::U][S::ROWS],
                                          unsigned long long* best = nullptr) {
    const int n_groups = gemv_groups<S>(a);
    if (FIRST) {
        float acc[S::ROWS];
#pragma unroll
        for (int r = 0; r < S::ROWS; r++) acc[r] = 0.f;
        gemv_compute<DT, S::ROWS, S::U>(pre, xs4, 0, lane, acc);
        gemv_group<DT, EPI, S, SC1>(a, g, lane, xs4, acc, S::U, best);
        g += total_waves;
    }
    for (; g < n_groups; g += total_waves) {
        float acc[S::ROWS];
#pragma unroll
        for (int r = 0; r < S::ROWS; r++) acc[r] = 0.f;
        gemv_group<DT, EPI, S, SC1>(a, g, lane, xs4, acc, 0, best);
    }
}

// PIPE 2: the wave's groups g, g + total_waves, ... as ONE stream of U-chunk steps (n has whole
// steps only).  Each step's chunks go into one of two register sets, and the NEXT step's
// chunks (the next group's first ones at a group end) are requested before the current set is
// multiplied, so a wave keeps U to 2U chunks per row in flight instead of draining to zero at
// every step, and a group's reduction and epilogue run behind the next group's loads.
// FIRST: the first group's step 0 is already in `pre`.
// gguf blocks (GQ): every step also loads its chunks' block scales (a second register set),
// and `pre_d` holds the first step's scales.
template <int DT, int EPI, class S, bool FIRST, bool SC1 = false>
__device__ __forceinline__ void gemv_rows_pipe(const GemvArgs& a, const int g0, const int total_waves, const int lane,
                                               const float4* xs4, const u32x4 (&pre)[S::U][S::ROWS],
                                               unsigned long long* best = nullptr,
                                               const float (*pre_d)[S::ROWS] = nullptr) {
    constexpr int ROWS = S::ROWS, U = S::U;
    constexpr int E = WDec<DT>::E;
    constexpr bool GQ = WScale<DT>::BLOCK > 0;
    const int n_groups = gemv_groups<S>(a);
    if (g0 >= n_groups) return;
    const int steps = a.n / (64 * E * U);
    const size_t qb = GQ ? gq_qbytes(DT, (size_t)a.n) : 0;
    // step k of this wave: group g0 + (k / steps) * total_waves, chunks from (k % steps) * U
    const int total = ((n_groups - g0 + total_waves - 1) / total_waves) * steps;
    // QKV: requested with the weights, ahead of the epilogue that uses them.  One-byte weights
    // only: fp8 decode 596 -> 603 tok/s, while the 2-byte qkv launch measured 0.5 % slower with it
    // (same-box A/B, two pairs each; again with the rope table: 393.3 vs 391.2 tok/s, 3 pairs)
    constexpr bool QKV = EPI == EPI_QKV && E >= 16;
    QkvPre<ROWS> qp{};
    if constexpr (QKV) {
        qp.pos = a.sp->pos;
        qp.kv_pos = a.sp->kv_pos;
    }
    // QKV: the rotation (cos, sin) of each row pair of the step's group; RESID: its residual rows
    constexpr bool RES = EPI == EPI_RESID && !SC1;
    float fa[ROWS], fb[ROWS];
    auto load = [&](u32x4 (&w)[U][ROWS], float (&d)[U][ROWS], float (&f)[ROWS], const int k) {
        const int q = k / steps;
        size_t rs;
        const char* wrow = gemv_row_ptr<ROWS>(a, g0 + q * total_waves, lane, rs);
        gemv_load<ROWS, U, S::NT>(w, wrow, rs, (k - q * steps) * U);
        if constexpr (GQ) gq_load_scales<DT, ROWS, U>(d, wrow, rs, qb, (k - q * steps) * U, lane);
        if constexpr (QKV) {
            const int row0 = min((g0 + q * total_waves) * ROWS, a.rows - ROWS);
#pragma unroll
            for (int p = 0; p < ROWS; p += 2) {
                const int j = ((row0 + p) % a.head_dim) >> 1;
                f[p] = a.rope_cs[j];
                f[p + 1] = a.rope_cs[(a.head_dim >> 1) + j];
            }
        }
        if constexpr (RES) {
            const int row0 = (g0 + q * total_waves) * ROWS;
#pragma unroll
            for (int r = 0; r < ROWS; r++) f[r] = a.out[min(row0 + r, a.rows - 1)];
        }
    };
    float acc[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; r++) acc[r] = 0.f;
    // multiply step k's chunks; after a group's last step, its reduction and epilogue
    auto step = [&](const u32x4 (&w)[U][ROWS], const float (&d)[U][ROWS], const float (&f)[ROWS], const int k) {
        const int q = k / steps;
        const int it = (k - q * steps) * U;
        if constexpr (GQ) gq_compute<DT, ROWS, U>(w, d, xs4, it, lane, acc, gq4_image<DT>() ? gq4_nxs(xs4, a.n) : nullptr);
        else gemv_compute<DT, ROWS, U>(w, xs4, it, lane, acc);
        if (it + U == steps * U) {
#pragma unroll
            for (int r = 0; r < ROWS; r++) acc[r] = wave_sum(acc[r]);
            if constexpr (QKV) {
#pragma unroll
                for (int p = 0; p < ROWS; p++) qp.cs[p] = f[p];
            }
            if (lane == 0)
                gemv_epilogue<EPI, ROWS, SC1>(a, (g0 + q * total_waves) * ROWS, acc, best, QKV ? &qp : nullptr,
                                              RES ? f : nullptr);
#pragma unroll
            for (int r = 0; r < ROWS; r++) acc[r] = 0.f;
        }
    };
    u32x4 wa[U][ROWS], wb[U][ROWS];
    float da[U][ROWS], db[U][ROWS];  // GQ only (otherwise unused)
    if constexpr (FIRST) {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < ROWS; r++) {
                wa[u][r] = pre[u][r];
                if constexpr (GQ) da[u][r] = pre_d[u][r];
            }
        if constexpr (QKV) {
            const int row0 = min(g0 * ROWS, a.rows - ROWS);
#pragma unroll
            for (int p = 0; p < ROWS; p += 2) {
                const int j = ((row0 + p) % a.head_dim) >> 1;
                fa[p] = a.rope_cs[j];
                fa[p + 1] = a.rope_cs[(a.head_dim >> 1) + j];
            }
        }
        if constexpr (RES) {
#pragma unroll
            for (int r = 0; r < ROWS; r++) fa[r] = a.out[min(g0 * ROWS + r, a.rows - 1)];
        }
    } else {
        load(wa, da, fa, 0);
    }
    // the loads stay outside any branch, so the compiler's waits count only the older set
    int k = 0;
    for (; k + 2 < total; k += 2) {
        load(wb, db, fb, k + 1);
        step(wa, da, fa, k);
        load(wa, da, fa, k + 2);
        step(wb, db, fb, k + 1);
    }
    if (k + 1 < total) {
        load(wb, db, fb, k + 1);
        step(wa, da, fa, k);
        step(wb, db, fb, k + 1);
    } else {
        step(wa, da, fa, k);
    }
}

// PF staging, part 1: this thread's x float4s (and norm weights) into registers.  Issued
// BEFORE the weight prefetch, so waiting for them (vmcnt counts in issue order) leaves the
// weight chunks in flight.
template <int PRO, class S>
__device__ __forceinline__ void stage_x_issue(const GemvArgs& a, float4 (&xv)[S::XN], float4 (&nw)[S::XN]) {
    const int n4 = a.n >> 2;
    const float4* x4 = (const float4*)a.x;
    // clamped indices, no branches: every load of the prologue sits in one basic block, so the
    // waits for x count only the x loads (threads past n4 reload the last float4; unused)
#pragma unroll
    for (int j = 0; j < S::XN; j++) {
        const int i = min((int)threadIdx.x + j * S::THREADS, n4 - 1);
        xv[j] = x4[i];
        if (PRO != PRO_PLAIN) nw[j] = load_norm4_nb(a.norm_w, a.norm_dtype, a.n, i);
    }
}
// part 2: rms scale (same per-thread order, shuffle tree and wave order as block_rms_scale, so
// the same value) and the permuted LDS image.  Branch-free like part 1 (a branch would let the
// compiler sink a load to its use and wait for the weights too): clamped duplicates are
// masked out of the sum and store the same value to the same slot.
template <int E, int PRO, class S, bool GQ4 = false>
__device__ __forceinline__ void stage_x_finish(const GemvArgs& a, const float4 (&xv)[S::XN], const float4 (&nw)[S::XN],
                                               float4* xs4, float* red) {
    const int n4 = a.n >> 2;
    float scale = 1.f;
    if (PRO != PRO_PLAIN) {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < S::XN; j++) {
            const float4 v = xv[j];
            const float d = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
            ss += ((int)threadIdx.x + j * S::THREADS < n4) ? d : 0.f;
        }
        ss = wave_sum(ss);
#ifdef GEMV_TRACE_X
        if (a.trace && threadIdx.x == GEMV_TRACE_X * 64) a.trace[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime();  // x landed (that wave)
#endif
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < S::WAVES; w++) tot += red[w];
        scale = 1.0f / sqrtf(tot / (float)a.n + a.eps);
    }
#ifdef GEMV_TRACE_X
    if (PRO == PRO_PLAIN && a.trace && threadIdx.x == GEMV_TRACE_X * 64) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < S::XN; j++) t += xv[j].x;  // waits for this thread's x loads
        a.trace[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime() + (t == 12345.f ? 1 : 0);
    }
#endif
#pragma unroll
    for (int j = 0; j < S::XN; j++) {
        const int i = min((int)threadIdx.x + j * S::THREADS, n4 - 1);
        float4 v = xv[j];
        if (PRO != PRO_PLAIN) {
            v.x = v.x * scale * nw[j].x;  // x[i] * scale * weight[i], src/infer.cpp:234
            v.y = v.y * scale * nw[j].y;
            v.z = v.z * scale * nw[j].z;
            v.w = v.w * scale * nw[j].w;
        }
        if constexpr (GQ4) v = gq4_stage(v, i, (int)threadIdx.x + j * S::THREADS < n4, xs4, a.n);
        const int c = i << 2;
        const int it = c / (64 * E);
        const int rem = c - it * 64 * E;
        const int l = rem / E;
        const int qd = (rem - l * E) >> 2;
        xs4[(it * (E / 4) + qd) * 64 + l] = v;
    }
}

// The whole matvec of one workgroup: block / n_blocks are its index and the count among the
// workgroups that run this matvec (gemv_kernel: blockIdx.x / gridDim.x).  SC1: outputs stored
// write-through (for a consumer inside the same launch).
template <int DT, int PRO, int EPI, class S, bool SC1 = false>
__device__ __forceinline__ void gemv_body(const GemvArgs& a, const int block, const int n_blocks, char* smem) {
    float* red = (float*)smem;
    float4* xs4 = (float4*)(smem + LDS_HEAD_BYTES);
    constexpr int E = WDec<DT>::E;
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    // BAL: wave-major group order (g = wid * n_blocks + block), so the groups past the last one
    // fall on the same waves of every workgroup and each CU gets the same share
    const int g = S::BAL ? wid * n_blocks + block : block * S::WAVES + wid;
#ifdef GEMV_TRACE_START
    if (a.trace && threadIdx.x == GEMV_TRACE_START * 64) a.trace[4 * block + 3] = __builtin_amdgcn_s_memrealtime();
#endif
    if (a.trace && threadIdx.x == 0) {
        a.trace[4 * block] = __builtin_amdgcn_s_memrealtime();
#if !defined(GEMV_TRACE_X) && !defined(GEMV_TRACE_START)
        unsigned xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 3)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        a.trace[4 * block + 3] = ((unsigned long long)xcc << 32) | hw;  // XCD, HW_ID (CU / SE bits)
#endif
    }
    if (a.aw_reset && block == 0 && threadIdx.x < AW_RESET_WORDS) a.aw_reset[32 * threadIdx.x] = 0u;
    unsigned long long best = 0;  // EPI_LOGITS: this wave's best candidate (lane 0)

    // gguf blocks: the pipelined PF shapes (block scales loaded beside the codes), else staged
    if constexpr (S::PF && (WScale<DT>::BLOCK == 0 || S::PIPE == 2)) {
        float4 xv[S::XN], nw[S::XN];
        stage_x_issue<PRO, S>(a, xv, nw);
        // unconditional (a wave past the last group re-reads that group's chunks, unused)
        const int n_groups = gemv_groups<S>(a);
        const bool prefetched = g < n_groups;
        u32x4 pre[S::U][S::ROWS];
        float pre_d[S::U][S::ROWS];
        gemv_prefetch<S>(a, min(g, n_groups - 1), lane, pre);
        if constexpr (WScale<DT>::BLOCK > 0) {
            size_t rs;
            const char* wrow = gemv_row_ptr<S::ROWS>(a, min(g, n_groups - 1), lane, rs);
            gq_load_scales<DT, S::ROWS, S::U>(pre_d, wrow, rs, gq_qbytes(DT, (size_t)a.n), 0, lane);
        }
        stage_x_finish<E, PRO, S, gq4_image<DT>()>(a, xv, nw, xs4, red);
        if (EPI == EPI_QKV && block == 0) rotate_sinks<S::THREADS>(a, a.sp->kv_sink);
        __syncthreads();
        if (a.trace && threadIdx.x == 0) a.trace[4 * block + 1] = __builtin_amdgcn_s_memrealtime();
        if constexpr (S::PIPE == 2) {
            if (prefetched) gemv_rows_pipe<DT, EPI, S, true, SC1>(a, g, n_blocks * S::WAVES, lane, xs4, pre, &best, pre_d);
        } else {
            if (prefetched) gemv_rows<DT, EPI, S, true, SC1>(a, g, n_blocks * S::WAVES, lane, xs4, pre, &best);
            else gemv_rows<DT, EPI, S, false, SC1>(a, g, n_blocks * S::WAVES, lane, xs4, pre, &best);
        }
    } else {
        stage_x<E, PRO, S::THREADS, false, gq4_image<DT>()>(a, xs4, red);
        if (EPI == EPI_QKV && block == 0) rotate_sinks<S::THREADS>(a, a.sp->kv_sink);
        __syncthreads();
        if (a.trace && threadIdx.x == 0) a.trace[4 * block + 1] = __builtin_amdgcn_s_memrealtime();
        u32x4 none[S::U][S::ROWS];
        if constexpr (S::PIPE == 2 && WScale<DT>::BLOCK == 0)
            gemv_rows_pipe<DT, EPI, S, false, SC1>(a, g, n_blocks * S::WAVES, lane, xs4, none, &best);
        else
            gemv_rows<DT, EPI, S, false, SC1>(a, g, n_blocks * S::WAVES, lane, xs4, none, &best);
    }
    if constexpr (EPI == EPI_LOGITS) {
        // the workgroup's candidate: lane 0 of each wave holds its best
        unsigned long long* kb = (unsigned long long*)smem;  // the rms scratch is free again
        __syncthreads();
        if (lane == 0) kb[wid] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long bb = 0;
#pragma unroll
            for (int w = 0; w < S::WAVES; w++) bb = kb[w] > bb ? kb[w] : bb;
            a.cand[block] = bb;
        }
    }
    if (a.trace) {
        __syncthreads();
        if (threadIdx.x == 0) a.trace[4 * block + 2] = __builtin_amdgcn_s_memrealtime();
    }
}

template <int DT, int PRO, int EPI, class S>
__global__ __launch_bounds__(S::THREADS, S::MINW) void gemv_kernel(const GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    gemv_body<DT, PRO, EPI, S>(a, blockIdx.x, gridDim.x, smem);
}

// LDS bytes and grid of one launch
template <int DT, class S>
inline size_t gemv_smem_bytes(const int n) {
    constexpr int E = WDec<DT>::E;
    const int n_it = (n + 64 * E - 1) / (64 * E);
    // Q4_0: -8 sum(x) per 32-element block after the image (gq4_nxs)
    return LDS_HEAD_BYTES + (size_t)n_it * 64 * E * sizeof(float) + (gq4_image<DT>() ? (size_t)n_it * 64 * sizeof(float) : 0);
}
// balanced rounds: at most max_blocks * WAVES waves, each with the same group count
template <class S>
inline int gemv_blocks(const int rows, const int max_blocks) {
    const int n_groups = (rows + S::ROWS - 1) / S::ROWS;
    const int w_max = max_blocks * S::WAVES;
    const int rounds = (n_groups + w_max - 1) / w_max;
    const int waves = (n_groups + rounds - 1) / rounds;
    const int blocks = (waves + S::WAVES - 1) / S::WAVES;
    // BAL: whole multiples of the CU count, so every CU holds the same number of workgroups
    // (448 blocks of 8 waves put 2 on 192 CUs and 1 on 64)
    if (S::BAL && blocks > GEMV_BAL_CU / 2) {
        const int up = (blocks + GEMV_BAL_CU - 1) / GEMV_BAL_CU * GEMV_BAL_CU;
        if (up <= max_blocks) return up;
    }
    return blocks;
}

}  // namespace xalm
