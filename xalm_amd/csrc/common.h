// common.h — device-side element decode and wave/block reductions for gfx950.
//
// Decode semantics are the reference's (jubruckne/Xalm src/types.h), bit for bit:
//   f16   : IEEE binary16 -> f32 (ARM float16_t promotion)
//   bf16  : bits << 16                                   (bf16_to_f32, src/types.h:322-325)
//   e4m3  : ((b&0x80)<<24 | (b&0x7f)<<20) * 2^120        (f8_t::to_float, src/types.h:302-314)
//   e5m2  : ((b&0x80)<<24 | (b&0x7f)<<21) * 2^112        (same, M=2)
//   q8    : (1.f/100.f) * (float)int8                    (Type::Q8, src/types.h:423-424)
// The fp8 bit forms equal OCP e4m3fn / e5m2 for every finite code and give the reference's
// finite values for the NaN/Inf codes (e4m3 0x7F -> 480), which the hardware converter would
// not: matrices use the converter unless they hold such a code (WDec<*_EXACT>).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/xalm_hip.h"

namespace xalm {

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
typedef float f2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // native vector: nontemporal loads

__device__ __forceinline__ float bits_f32(uint32_t u) { return __builtin_bit_cast(float, u); }

// 16 bytes of weights -> E floats.  E = 16 / sizeof(element).
template <int DT> struct WDec;

template <> struct WDec<XH_F32> {
    static constexpr int E = 4;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) {
        f[0] = bits_f32(v.x); f[1] = bits_f32(v.y); f[2] = bits_f32(v.z); f[3] = bits_f32(v.w);
    }
};

template <> struct WDec<XH_F16> {
    static constexpr int E = 8;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const f2_t p = __builtin_convertvector(__builtin_bit_cast(h2_t, w[i]), f2_t);
            f[2 * i] = p.x;
            f[2 * i + 1] = p.y;
        }
    }
};

template <> struct WDec<XH_BF16> {
    static constexpr int E = 8;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            f[2 * i] = bits_f32(w[i] << 16);
            f[2 * i + 1] = bits_f32(w[i] & 0xffff0000u);
        }
    }
};

template <int SHIFT, int SCALE_EXP>
__device__ __forceinline__ void dec_f8_word(const uint32_t w, float* f) {
    // byte k of w -> sign to bit 31, low 7 bits to the top of the f32 exponent field
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t b = (w >> (8 * k)) & 0xffu;
        const uint32_t u = ((b & 0x80u) << 24) | ((b & 0x7fu) << SHIFT);
        f[k] = bits_f32(u) * __builtin_bit_cast(float, (uint32_t)((127 + SCALE_EXP) << 23));
    }
}

// fp8 with the gfx950 converter (v_cvt_pk_f32_fp8 / _bf8: OCP e4m3fn / e5m2, 2 elements per
// instruction).  Equal to the reference's bit form for every code except the NaN/Inf codes
// (e4m3 0x7F/0xFF; e5m2 exponent 31), which the host detects at upload: a matrix holding
// any of them is decoded with the *_EXACT forms below instead.
template <bool BF8>
__device__ __forceinline__ void dec_f8_hw(const u32x4 v, float* f) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const f2_t lo = BF8 ? __builtin_amdgcn_cvt_pk_f32_bf8(w[i], false) : __builtin_amdgcn_cvt_pk_f32_fp8(w[i], false);
        const f2_t hi = BF8 ? __builtin_amdgcn_cvt_pk_f32_bf8(w[i], true) : __builtin_amdgcn_cvt_pk_f32_fp8(w[i], true);
        f[4 * i + 0] = lo.x;
        f[4 * i + 1] = lo.y;
        f[4 * i + 2] = hi.x;
        f[4 * i + 3] = hi.y;
    }
}
template <> struct WDec<XH_F8_E4M3> {
    static constexpr int E = 16;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) { dec_f8_hw<false>(v, f); }
};
template <> struct WDec<XH_F8_E5M2> {
    static constexpr int E = 16;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) { dec_f8_hw<true>(v, f); }
};

// internal kernel dtypes: fp8 matrices that hold NaN/Inf codes, decoded bit-exactly as the
// reference (f8_t::to_float, src/types.h:302-314: finite values for every code)
constexpr int XH_F8_E4M3_EXACT = 106;
constexpr int XH_F8_E5M2_EXACT = 107;
template <> struct WDec<XH_F8_E4M3_EXACT> {
    static constexpr int E = 16;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) {
        dec_f8_word<20, 120>(v.x, f);
        dec_f8_word<20, 120>(v.y, f + 4);
        dec_f8_word<20, 120>(v.z, f + 8);
        dec_f8_word<20, 120>(v.w, f + 12);
    }
};
template <> struct WDec<XH_F8_E5M2_EXACT> {
    static constexpr int E = 16;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) {
        dec_f8_word<21, 112>(v.x, f);
        dec_f8_word<21, 112>(v.y, f + 4);
        dec_f8_word<21, 112>(v.z, f + 8);
        dec_f8_word<21, 112>(v.w, f + 12);
    }
};
// the code's NaN/Inf pattern under OCP (where the hardware converter and the reference differ)
__host__ __device__ inline bool f8_special(const uint8_t b, const bool e5m2) {
    return e5m2 ? (b & 0x7Cu) == 0x7Cu : (b & 0x7Fu) == 0x7Fu;
}

template <> struct WDec<XH_Q8> {
    static constexpr int E = 16;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int8_t q = (int8_t)((w[i] >> (8 * k)) & 0xffu);
                f[4 * i + k] = (1.f / 100.f) * (float)q;
            }
    }
};

// ---- gguf blocks (XH_Q8_0, XH_Q4_0; quants.py Q8_0 :438-454, Q4_0 :281-311) --------------
// Device rows are planar: [quant bytes][f16 scale per 32 elements], pitch a multiple of 16 B,
// so a 16-B load is 16 int8 (Q8_0, half a block) or 32 nibbles (Q4_0, one block) and the
// scales of a wave's chunks are one coalesced read.  WDec decodes the codes (q, q - 8); the
// matvec multiplies each chunk's partial dot product by its block's d.
__host__ __device__ constexpr bool gq_dt(const int dt) { return dt == XH_Q8_0 || dt == XH_Q4_0; }
__host__ __device__ constexpr size_t gq_qbytes(const int dt, const size_t n) { return dt == XH_Q8_0 ? n : n / 2; }
__host__ __device__ constexpr size_t gq_pitch(const int dt, const size_t n) {
    return (gq_qbytes(dt, n) + n / 16 + 15) & ~(size_t)15;
}
__host__ __device__ constexpr size_t gq_block_bytes(const int dt) { return dt == XH_Q8_0 ? 34 : 18; }
template <int DT> struct WScale { static constexpr int BLOCK = 0; };  // elements per scale (0: none)
template <> struct WScale<XH_Q8_0> { static constexpr int BLOCK = 32; };
template <> struct WScale<XH_Q4_0> { static constexpr int BLOCK = 32; };

template <> struct WDec<XH_Q8_0> {
    static constexpr int E = 16;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int k = 0; k < 4; k++) f[4 * i + k] = (float)(int8_t)((w[i] >> (8 * k)) & 0xffu);
    }
};
template <> struct WDec<XH_Q4_0> {
    static constexpr int E = 32;
    __device__ __forceinline__ static void dec(const u32x4 v, float* f) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t b = (w[i] >> (8 * k)) & 0xffu;
                f[4 * i + k] = (float)((int)(b & 15u) - 8);        // element j = 4i + k
                f[16 + 4 * i + k] = (float)((int)(b >> 4) - 8);    // element j + 16
            }
    }
};

// single-element decode (embedding gather, norm weights)
__device__ __forceinline__ float dec1(const int dtype, const void* p, const size_t i) {
    switch (dtype) {
        case XH_F32: return ((const float*)p)[i];
        case XH_F16: return (float)((const _Float16*)p)[i];
        case XH_BF16: return bits_f32((uint32_t)((const uint16_t*)p)[i] << 16);
        case XH_F8_E4M3: {
            const uint32_t b = ((const uint8_t*)p)[i];
            return bits_f32(((b & 0x80u) << 24) | ((b & 0x7fu) << 20)) * 0x1p120f;
        }
        case XH_F8_E5M2: {
            const uint32_t b = ((const uint8_t*)p)[i];
            return bits_f32(((b & 0x80u) << 24) | ((b & 0x7fu) << 21)) * 0x1p112f;
        }
        case XH_Q8: return (1.f / 100.f) * (float)((const int8_t*)p)[i];
        default: return __builtin_nanf("");
    }
}

// element i of row `row` of a [rows][n] matrix of `dtype` (gguf blocks: the planar device rows)
__device__ __forceinline__ float dec_row(const int dtype, const void* p, const size_t row, const int n, const int i) {
    if (!gq_dt(dtype)) return dec1(dtype, p, row * (size_t)n + i);
    const uint8_t* r = (const uint8_t*)p + row * gq_pitch(dtype, n);
    const float d = (float)__builtin_bit_cast(_Float16, *(const uint16_t*)(r + gq_qbytes(dtype, n) + (i >> 5) * 2));
    if (dtype == XH_Q8_0) return d * (float)(int8_t)r[i];
    const uint8_t b = r[(i >> 5) * 16 + (i & 15)];
    return d * (float)((int)((i & 16) ? (b >> 4) : (b & 15u)) - 8);
}

__device__ __forceinline__ uint16_t f32_to_f16_bits(const float f) {
    return __builtin_bit_cast(uint16_t, (_Float16)f);  // v_cvt_f16_f32, round-to-nearest-even
}
__device__ __forceinline__ float f16_bits_to_f32(const uint16_t h) {
    return (float)__builtin_bit_cast(_Float16, h);
}

// ---- cross-lane reductions without LDS: DPP within 16-lane rows, permlane swaps across rows
// (v_permlane16/32_swap, gfx950; hipcc inserts the VALU->permlane wait states).  Every lane of
// the reduced group ends with the same value.
enum { DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_ROW_ROR = 0x120, DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141 };
template <int CTRL>
__device__ __forceinline__ float dpp(const float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
struct OpSum { __device__ static float f(float a, float b) { return a + b; } };
struct OpMax { __device__ static float f(float a, float b) { return fmaxf(a, b); } };
// combine the two rows of each row pair (1 with 0, 3 with 2) / the two half-waves
// The swaps are inline asm: hipcc (ROCm 7.2) takes the builtins' second result from the
// first operand's register (measured: permlane16_swap(x, y)[1] came back equal to [0]).  The
// s_nop 1 covers the "VALU write -> v_permlane read" hazard (cdna_hip_programming.md T21).
template <class Op>
__device__ __forceinline__ float rows_pair(const float v) {
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return Op::f(a, b);
}
template <class Op>
__device__ __forceinline__ float halves(const float v) {
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return Op::f(a, b);
}
// over aligned groups of G consecutive lanes (G = 2, 4, ..., 64)
template <int G, class Op = OpSum>
__device__ __forceinline__ float group_reduce(float v) {
    if (G >= 2) v = Op::f(v, dpp<DPP_XOR1>(v));
    if (G >= 4) v = Op::f(v, dpp<DPP_XOR2>(v));
    if (G >= 8) v = Op::f(v, dpp<DPP_ROW_HALF_MIRROR>(v));
    if (G >= 16) v = Op::f(v, dpp<DPP_ROW_MIRROR>(v));
    if (G >= 32) v = rows_pair<Op>(v);
    if (G >= 64) v = halves<Op>(v);
    return v;
}
// over the 64 / S lanes congruent mod S (S = 1, 2, 4, ..., 32): lanes l, l+S, l+2S, ...
template <int S, class Op = OpSum>
__device__ __forceinline__ float strided_reduce(float v) {
    if (S <= 1) v = Op::f(v, dpp<DPP_ROW_ROR + 1>(v));
    if (S <= 2) v = Op::f(v, dpp<DPP_ROW_ROR + 2>(v));
    if (S <= 4) v = Op::f(v, dpp<DPP_ROW_ROR + 4>(v));
    if (S <= 8) v = Op::f(v, dpp<DPP_ROW_ROR + 8>(v));
    if (S <= 16) v = rows_pair<Op>(v);
    v = halves<Op>(v);
    return v;
}
// Reduce-scatter of N per-lane values over the four 16-lane rows of a wave: on return v[0, N/4)
// of every lane of row r holds the 4-row sums of values [(r & 1) * N/2 + (r >> 1) * N/4, + N/4)
// (N/2 + N/4 swaps instead of 2 N for a full all-reduce of every value).
template <int N>
__device__ __forceinline__ void rows_reduce_scatter(float (&v)[N]) {
    static_assert(N % 4 == 0, "N must be a multiple of 4");
    // each swap carries its own s_nop 1: the operands may be fresh VALU copies (T21 hazard)
#pragma unroll
    for (int k = 0; k < N / 2; k++) {
        float x = v[k], y = v[N / 2 + k];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
        v[k] = x + y;
    }
#pragma unroll
    for (int k = 0; k < N / 4; k++) {
        float x = v[k], y = v[N / 4 + k];
        asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
        v[k] = x + y;
    }
}

__device__ __forceinline__ float wave_sum(float v) { return group_reduce<64, OpSum>(v); }
__device__ __forceinline__ float wave_max(float v) { return group_reduce<64, OpMax>(v); }

// Orderable key of (logit, index) for Sampler::sample_argmax (src/sampler.cpp:19-30): a larger
// logit wins, then the smaller index (the first maximum); 0 = no candidate.
__device__ __forceinline__ unsigned long long argmax_key(const float v, const int idx) {
    uint32_t u = __builtin_bit_cast(uint32_t, v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (uint32_t)(~(uint32_t)idx);
}
__device__ __forceinline__ int argmax_key_index(const unsigned long long k) { return k ? (int)(~(uint32_t)k) : 0; }

// Per-token dynamic scalars, read by every kernel of a captured graph.
// kv_sink / kv_pos / kv_len follow src/infer.cpp:611-613.
struct StepParams {
    int token;
    int pos;
    int kv_sink;
    int kv_pos;
    int kv_len;
    int step;      // device decode loop: index into the token output buffer
    int pos_next;  // device decode loop: position of the next forward
    int max_seq_len;
};

__device__ __forceinline__ void step_positions(StepParams* sp, const int pos) {
    const int msl = sp->max_seq_len;
    const int kv_sink = pos >= msl ? 2 : 0;  // KV_SINKS, src/model.h:10
    sp->pos = pos;
    sp->kv_sink = kv_sink;
    sp->kv_pos = kv_sink + (pos - kv_sink) % (msl - kv_sink);
    sp->kv_len = pos >= msl ? msl : pos + 1;
}

// 16-byte sc1 load through a buffer descriptor (aux 16 = sc1, cdna_hip_programming.md T8 / G16)
__device__ __forceinline__ u32x4 ld_sc1_x4(const void* base, const uint32_t byte_off) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)byte_off, 0, 16));
}

// silu / gelu exactly as src/infer.cpp:299-301
__device__ __forceinline__ float act_fn(const int act, const float x) {
    if (act == XH_ACT_SILU) return x / (1.0f + expf(-x));
    return 0.5f * x * (1.0f + tanhf(0.797885f * (x + 0.044715f * x * x * x)));
}

}  // namespace xalm
