/*
 * xalm_synth.h — deterministic synthetic weights for benchmarks (no checkpoints offline).
 *
 * One definition, compiled by gcc (oracle / CPU baseline) and by hipcc (device fill kernel),
 * so a tensor generated on the GPU is bit-identical to the host copy the CPU baseline uses.
 * Value of element i: mean + std * sqrt(3) * (u0 + u1 + u2 + u3 - 2), u_k uniform [0,1) from
 * a splitmix64 hash of (seed, i, k) (Irwin-Hall, variance 1/3 -> scaled to 1): integer ops,
 * float adds and one explicit fmaf only, so no libm or contraction differences between
 * compilers.  Then rounded to the storage type with round-to-nearest-even (f16, bf16, and
 * OCP e4m3 / e5m2 with subnormals, saturating to the max finite value as a safety net).
 */
#ifndef XALM_SYNTH_H
#define XALM_SYNTH_H

#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#define XS_FN __host__ __device__ static inline
#else
#define XS_FN static inline
#endif

XS_FN uint64_t xs_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

XS_FN float xs_u01(uint64_t h) { return (float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f); }

XS_FN float xs_value(uint64_t seed, uint64_t i, float mean, float std) {
    const uint64_t h0 = xs_mix(seed ^ (i * 0xD1B54A32D192ED03ull));
    const uint64_t h1 = xs_mix(h0);
    const float u0 = xs_u01(h0), u1 = xs_u01(h0 << 24), u2 = xs_u01(h1), u3 = xs_u01(h1 << 24);
    const float s = ((u0 + u1) + (u2 + u3)) - 2.0f;
    return fmaf(s, std * 1.7320508f, mean);
}

XS_FN uint32_t xs_f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
XS_FN float xs_bits_f32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* float -> bf16, RNE (finite inputs) */
XS_FN uint16_t xs_to_bf16(float f) {
    const uint32_t u = xs_f32_bits(f);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

/* float -> IEEE half, RNE, finite inputs with |f| < 65504 (synthetic weights are small) */
XS_FN uint16_t xs_to_f16(float f) {
    const uint32_t x = xs_f32_bits(f);
    const uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    const uint32_t a = x & 0x7FFFFFFFu;
    if (a >= 0x477FF000u) return (uint16_t)(sign | 0x7BFFu);          /* saturate */
    if (a < 0x38800000u) {                                            /* half subnormal / zero */
        const float m = xs_bits_f32(a) * 16777216.0f;                 /* |f| * 2^24, exact */
        /* RNE to integer without libm: add and subtract 2^23 */
        const float r = (m + 8388608.0f) - 8388608.0f;
        return (uint16_t)(sign | (uint16_t)r);
    }
    uint32_t m = a + 0xC8000000u;                                     /* rebias exponent 127 -> 15 */
    m = m + 0x0FFFu + ((m >> 13) & 1u);
    return (uint16_t)(sign | (uint16_t)(m >> 13));
}

/* float -> OCP fp8 with E exponent bits (4 or 5), M = 7 - E mantissa bits; RNE with
 * subnormals; saturates to the largest finite code (never produces NaN / Inf codes). */
XS_FN uint8_t xs_to_f8(float f, int E) {
    const int M = 7 - E;
    const int bias = (1 << (E - 1)) - 1;
    const uint32_t x = xs_f32_bits(f);
    const uint8_t sign = (uint8_t)((x >> 24) & 0x80u);
    const float a = xs_bits_f32(x & 0x7FFFFFFFu);
    const uint8_t maxcode = E == 4 ? 0x7E : 0x7B;
    const float maxval = E == 4 ? 448.0f : 57344.0f;
    if (!(a < maxval)) return (uint8_t)(sign | maxcode);
    const float min_normal = xs_bits_f32((uint32_t)(127 + 1 - bias) << 23);
    if (a < min_normal) {
        /* subnormal: value = q * 2^(1-bias-M), q in [0, 2^M]; RNE via 2^23 trick */
        const float scale = xs_bits_f32((uint32_t)(127 - (1 - bias - M)) << 23);
        const float q = (a * scale + 8388608.0f) - 8388608.0f;
        return (uint8_t)(sign | (uint8_t)q);  /* q == 2^M rolls into the first normal code */
    }
    uint32_t u = xs_f32_bits(a);
    const int sh = 23 - M;
    u = u + ((1u << (sh - 1)) - 1u) + ((u >> sh) & 1u);
    const int e = (int)(u >> 23) - 127 + bias;
    const uint32_t mant = (u >> sh) & ((1u << M) - 1u);
    uint32_t code = ((uint32_t)e << M) | mant;
    if (code > maxcode) code = maxcode;
    return (uint8_t)(sign | code);
}

/* ---- gguf blocks (XH_Q8_0 / XH_Q4_0): quantize 32 floats into one block of the converter's
 * file layout, restating quants.py (Q8_0.quantize_blocks :438-454, Q4_0.quantize_blocks
 * :283-299) with numpy's float32 semantics: a float32 op per numpy op, float16 by RNE,
 * np_roundf = round half away from zero, Q4_0's `trunc(float64(x) * float64(id) + 8.5)`
 * cast to float32 (the product of two floats is exact in double, so contraction cannot
 * change it). */
XS_FN float xs_roundf_away(float v) {
    const float a = fabsf(v);
    const float fl = floorf(a);
    const float b = fl + floorf(2.0f * (a - fl));
    return v < 0.0f ? -b : (v > 0.0f ? b : 0.0f * v);
}
/* out: 34 bytes, f16 d then 32 int8 */
XS_FN void xs_quant_q8_0(const float* v, uint8_t* out) {
    float amax = 0.0f;
    for (int k = 0; k < 32; k++) amax = fmaxf(amax, fabsf(v[k]));
    const float d = amax / 127.0f;
    const float id = d == 0.0f ? 0.0f : 1.0f / d;
    const uint16_t dh = xs_to_f16(d);
    out[0] = (uint8_t)(dh & 0xFFu);
    out[1] = (uint8_t)(dh >> 8);
    for (int k = 0; k < 32; k++) out[2 + k] = (uint8_t)(int8_t)xs_roundf_away(v[k] * id);
}
/* out: 18 bytes, f16 d then 16 bytes: byte j = q[j] | q[j+16] << 4 */
XS_FN void xs_quant_q4_0(const float* v, uint8_t* out) {
    int imax = 0;
    float amax = fabsf(v[0]);
    for (int k = 1; k < 32; k++)
        if (fabsf(v[k]) > amax) { amax = fabsf(v[k]); imax = k; }  /* argmax: the first maximum */
    const float d = v[imax] / -8.0f;
    const float id = d == 0.0f ? 0.0f : 1.0f / d;
    uint8_t q[32];
    for (int k = 0; k < 32; k++) {
        const float t = truncf((float)((double)v[k] * (double)id + 8.5));
        q[k] = (uint8_t)(t < 0.0f ? 0.0f : (t > 15.0f ? 15.0f : t));
    }
    const uint16_t dh = xs_to_f16(d);
    out[0] = (uint8_t)(dh & 0xFFu);
    out[1] = (uint8_t)(dh >> 8);
    for (int j = 0; j < 16; j++) out[2 + j] = (uint8_t)(q[j] | (q[j + 16] << 4));
}
/* synthetic block b of row r of a [rows][cols] tensor: the 32 values xs_value gives elements
 * r*cols + 32b .. +31, quantized (dtype 20 Q8_0 / 21 Q4_0) */
XS_FN void xs_block(uint8_t* out, int dtype, uint64_t seed, uint64_t r, uint64_t cols, uint64_t b, float mean, float std) {
    float v[32];
    for (int k = 0; k < 32; k++) v[k] = xs_value(seed, r * cols + 32 * b + k, mean, std);
    if (dtype == 20) xs_quant_q8_0(v, out);
    else xs_quant_q4_0(v, out);
}

/* dtype ids as in xalm_hip.h: 1 F32, 2 F16, 3 BF16, 6 F8_E4M3, 7 F8_E5M2 */
XS_FN void xs_store(void* dst, uint64_t idx, int dtype, float v) {
    switch (dtype) {
        case 1: ((float*)dst)[idx] = v; break;
        case 2: ((uint16_t*)dst)[idx] = xs_to_f16(v); break;
        case 3: ((uint16_t*)dst)[idx] = xs_to_bf16(v); break;
        case 6: ((uint8_t*)dst)[idx] = xs_to_f8(v, 4); break;
        case 7: ((uint8_t*)dst)[idx] = xs_to_f8(v, 5); break;
        default: break;
    }
}

#endif
