/*
 * xalm_oracle.c — CPU restatement of jubruckne/Xalm's forward pass (TEST INFRASTRUCTURE).
 *
 * Every function cites the reference file:line it restates.  Semantics follow the ARM
 * build the reference targets (bf16 norm weights are decoded to f32).
 * This file is the checker for the HIP path and the timed `-d cpu` baseline; nothing in
 * the product links it (see xalm_oracle.h).
 *
 * Build: oracle/Makefile  (gcc -O3 -fopenmp -mavx2 -mfma -mf16c; AVX-512 forms picked at run time)
 */
#include "xalm_oracle.h"

#include <float.h>
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#if defined(__F16C__) && defined(__AVX2__) && defined(__FMA__)
#include <immintrin.h>
#define XO_SIMD 1
#endif

#include "../include/xalm_synth.h"

#define KV_SINKS 2 /* src/model.h:10 */

/* Host copy of the device synthetic weights (xh_upload_synthetic): same header, same bits.
 * dst is a dense [rows][cols] tensor of `dtype`. */
void xo_fill_synthetic(void* dst, size_t rows, size_t cols, int dtype, uint64_t seed, float mean, float std) {
    const size_t n = rows * cols;
    size_t i;
    if (dtype == XH_Q8_0 || dtype == XH_Q4_0) {
        /* gguf blocks in the converter's file layout: [rows][cols/32 blocks] */
        const size_t nb = cols / 32, bs = dtype == XH_Q8_0 ? 34 : 18;
#pragma omp parallel for schedule(static)
        for (i = 0; i < rows * nb; i++) xs_block((uint8_t*)dst + i * bs, dtype, seed, i / nb, cols, i % nb, mean, std);
        return;
    }
#pragma omp parallel for schedule(static)
    for (i = 0; i < n; i++) xs_store(dst, i, dtype, xs_value(seed, i, mean, std));
}

/* ------------------------------------------------------------------------------------ */
/* element decode, src/types.h                                                          */
/* ------------------------------------------------------------------------------------ */
static inline float bits_f32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* IEEE binary16 -> binary32 (exact). ARM `float16_t` promotion. */
float xo_f16_to_f32(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16;
    const uint32_t e = (h >> 10) & 0x1fu;
    const uint32_t m = h & 0x3ffu;
    if (e == 0) {
        if (m == 0) return bits_f32(s);
        const float v = (float)m * 5.9604644775390625e-08f; /* m * 2^-24, exact */
        return s ? -v : v;
    }
    if (e == 31) return bits_f32(s | 0x7f800000u | (m << 13));
    return bits_f32(s | ((e + 112u) << 23) | (m << 13));
}

/* binary32 -> binary16, round to nearest even (ARM fcvt; the KV-cache store
 * `kb[...] = s.k()[i]`, src/infer.cpp:410-414). */
uint16_t xo_f32_to_f16(float fv) {
    const uint32_t f = f32_bits(fv);
    const uint16_t h_sgn = (uint16_t)((f & 0x80000000u) >> 16);
    uint32_t f_exp = f & 0x7f800000u;
    uint32_t f_sig;
    if (f_exp >= 0x47800000u) {
        if (f_exp == 0x7f800000u) {
            f_sig = f & 0x007fffffu;
            if (f_sig != 0) {
                uint16_t ret = (uint16_t)(0x7c00u + (f_sig >> 13));
                if (ret == 0x7c00u) ret++;
                return (uint16_t)(h_sgn + ret) | 0x0200u;
            }
        }
        return (uint16_t)(h_sgn + 0x7c00u);
    }
    if (f_exp <= 0x38000000u) {
        if (f_exp < 0x33000000u) return h_sgn;
        f_exp >>= 23;
        f_sig = 0x00800000u + (f & 0x007fffffu);
        f_sig >>= (113u - f_exp);
        if (((f_sig & 0x00003fffu) != 0x00001000u) || (f & 0x000007ffu)) f_sig += 0x00001000u;
        return (uint16_t)(h_sgn + (uint16_t)(f_sig >> 13));
    }
    const uint16_t h_exp = (uint16_t)((f_exp - 0x38000000u) >> 13);
    f_sig = f & 0x007fffffu;
    if ((f_sig & 0x00003fffu) != 0x00001000u) f_sig += 0x00001000u;
    return (uint16_t)(h_sgn + (uint16_t)((f_sig >> 13) + h_exp));
}

/* bf16_to_f32, src/types.h:322-325 */
static inline float bf16_to_f32(uint16_t h) { return bits_f32((uint32_t)h << 16); }

/* f8_t<E,M>::to_float, src/types.h:302-314: (sign<<24) | (bits&0x7F)<<(23-M), times
 * 2^(127-bias) with bias = 2^(E-1)-1. */
static inline float f8e4m3_to_f32(uint8_t b) {
    const uint32_t u = ((uint32_t)(b & 0x80u) << 24) | ((uint32_t)(b & 0x7fu) << 20);
    return bits_f32(u) * 0x1p120f;
}
static inline float f8e5m2_to_f32(uint8_t b) {
    const uint32_t u = ((uint32_t)(b & 0x80u) << 24) | ((uint32_t)(b & 0x7fu) << 21);
    return bits_f32(u) * 0x1p112f;
}
/* Type::Q8 get_float, src/types.h:423-424 */
static inline float q8_to_f32(int8_t q) { return (1.f / 100.f) * (float)q; }

float xo_decode(int dtype, const void* data, size_t idx) {
    switch (dtype) {
        case XH_F32: return ((const float*)data)[idx];
        case XH_F16: return xo_f16_to_f32(((const uint16_t*)data)[idx]);
        case XH_BF16: return bf16_to_f32(((const uint16_t*)data)[idx]);
        case XH_F8_E4M3: return f8e4m3_to_f32(((const uint8_t*)data)[idx]);
        case XH_F8_E5M2: return f8e5m2_to_f32(((const uint8_t*)data)[idx]);
        case XH_Q8: return q8_to_f32(((const int8_t*)data)[idx]);
        default: return NAN;
    }
}

/* gguf blocks, quants.py dequantize_blocks: Q8_0 (:448-454) x * d; Q4_0 (:302-311)
 * d * (nibble - 8), element j of a block in the low nibble of byte j (j < 16) or the high
 * nibble of byte j - 16; d the block's leading f16.  `row` of a [rows][n] tensor in the
 * converter's layout (n/32 blocks of 34 / 18 bytes per row). */
static inline int xo_gq(int dtype) { return dtype == XH_Q8_0 || dtype == XH_Q4_0; }
static inline size_t xo_gq_bs(int dtype) { return dtype == XH_Q8_0 ? 34 : 18; }
static inline float xo_gq_elem(int dtype, const uint8_t* blk, int k) {
    const float d = xo_f16_to_f32((uint16_t)(blk[0] | (blk[1] << 8)));
    if (dtype == XH_Q8_0) return (float)(int8_t)blk[2 + k] * d;
    const uint8_t b = blk[2 + (k & 15)];
    return d * (float)((int)(k < 16 ? (b & 15u) : (b >> 4)) - 8);
}
float xo_decode_row(int dtype, const void* data, size_t row, size_t n, size_t i) {
    if (!xo_gq(dtype)) return xo_decode(dtype, data, row * n + i);
    const uint8_t* blk = (const uint8_t*)data + (row * (n / 32) + i / 32) * xo_gq_bs(dtype);
    return xo_gq_elem(dtype, blk, (int)(i % 32));
}

/* the shared quantizer (include/xalm_synth.h, restating quants.py) over n_blocks blocks of 32
 * floats: the converter's block bytes (tests pin it against quants.py quantize) */
void xo_quantize_gq(int dtype, const float* v, size_t n_blocks, uint8_t* out) {
    for (size_t b = 0; b < n_blocks; b++) {
        if (dtype == XH_Q8_0) xs_quant_q8_0(v + 32 * b, out + 34 * b);
        else xs_quant_q4_0(v + 32 * b, out + 18 * b);
    }
}

static size_t dtype_bits(int dtype) {
    switch (dtype) {
        case XH_F32: return 32;
        case XH_F16: case XH_BF16: return 16;
        case XH_F8_E4M3: case XH_F8_E5M2: case XH_U8: case XH_Q8: return 8;
        default: return 0;
    }
}

/* ------------------------------------------------------------------------------------ */
/* ops, src/infer.cpp                                                                    */
/* ------------------------------------------------------------------------------------ */

/* matmul<TX,TW>, src/infer.cpp:104-135 (dispatch :185-216): xout[i] = sum_j dec(W[i,j])*x[j],
 * fp32 accumulate, OpenMP over rows (the reference's `omp simd` leaves the in-row order
 * implementation-defined; here 8-wide FMA lanes for f16). */
/* in-row summation order of the f16 matmul: 0 = 8-wide FMA lanes (default), 1 = sequential
 * (XO_MATMUL_SCALAR=1 or xo_set_matmul_order(1)); both are valid readings of the reference's
 * `omp simd` loop, so their difference measures the reference's own order sensitivity */
static int scalar_order = -1;
void xo_set_matmul_order(int order) { scalar_order = order != 0; }
int xo_matmul_order(void) {
    if (scalar_order < 0) scalar_order = getenv("XO_MATMUL_SCALAR") && atoi(getenv("XO_MATMUL_SCALAR"));
    return scalar_order;
}
#ifdef XO_SIMD
/* Row dot products in the "lanes" order: four 8-wide FMA accumulators over the column blocks
 * j, j+8, j+16, j+24 of every 32, summed (a0 + a1) + (a2 + a3), then horizontally, then the
 * tail sequentially.  The AVX-512 forms hold [a0 | a1] and [a2 | a3] in two 16-wide registers:
 * every lane sees the same FMAs in the same order, so both forms give the same bits; the host's
 * ISA is picked at run time (BASELINE.md §3 asks for -march=native; the library must also run
 * on hosts without AVX-512).  fp8 codes decode by the reference's bit formula (f8_t::to_float,
 * src/types.h:302-314), 8 or 16 at a time. */
static inline float hsum8(const __m256 a0, const __m256 a1, const __m256 a2, const __m256 a3) {
    const __m256 s = _mm256_add_ps(_mm256_add_ps(a0, a1), _mm256_add_ps(a2, a3));
    __m128 s4 = _mm_add_ps(_mm256_castps256_ps128(s), _mm256_extractf128_ps(s, 1));
    s4 = _mm_hadd_ps(s4, s4);
    s4 = _mm_hadd_ps(s4, s4);
    return _mm_cvtss_f32(s4);
}
static inline __m256 f8x8(const uint8_t* p, const int e5m2) {
    const __m256i b = _mm256_cvtepu8_epi32(_mm_loadl_epi64((const __m128i*)p));
    const __m256i sg = _mm256_slli_epi32(_mm256_and_si256(b, _mm256_set1_epi32(0x80)), 24);
    const __m256i mg = _mm256_and_si256(b, _mm256_set1_epi32(0x7f));
    const __m256i u = _mm256_or_si256(sg, e5m2 ? _mm256_slli_epi32(mg, 21) : _mm256_slli_epi32(mg, 20));
    return _mm256_mul_ps(_mm256_castsi256_ps(u), _mm256_set1_ps(e5m2 ? 0x1p112f : 0x1p120f));
}
/* one gguf block (quants.py dequantize_blocks, :302-311 / :448-454) as 4 x 8 f32: d * q exact
 * (q has <= 8 significant bits, d 11); element e of the block in lane e % 8 of register e / 8 */
static inline void gq_block8(const uint8_t* blk, const int dtype, __m256* v) {
    const __m256 d = _mm256_set1_ps(xo_f16_to_f32((uint16_t)(blk[0] | (blk[1] << 8))));
    if (dtype == XH_Q8_0) {
        for (int r = 0; r < 4; r++)
            v[r] = _mm256_mul_ps(_mm256_cvtepi32_ps(_mm256_cvtepi8_epi32(_mm_loadl_epi64((const __m128i*)(blk + 2 + 8 * r)))), d);
        return;
    }
    const __m128i b = _mm_loadu_si128((const __m128i*)(blk + 2));
    const __m128i lo = _mm_and_si128(b, _mm_set1_epi8(15)), hi = _mm_and_si128(_mm_srli_epi16(b, 4), _mm_set1_epi8(15));
    const __m256i m8 = _mm256_set1_epi32(8);
    v[0] = _mm256_mul_ps(_mm256_cvtepi32_ps(_mm256_sub_epi32(_mm256_cvtepu8_epi32(lo), m8)), d);
    v[1] = _mm256_mul_ps(_mm256_cvtepi32_ps(_mm256_sub_epi32(_mm256_cvtepu8_epi32(_mm_srli_si128(lo, 8)), m8)), d);
    v[2] = _mm256_mul_ps(_mm256_cvtepi32_ps(_mm256_sub_epi32(_mm256_cvtepu8_epi32(hi), m8)), d);
    v[3] = _mm256_mul_ps(_mm256_cvtepi32_ps(_mm256_sub_epi32(_mm256_cvtepu8_epi32(_mm_srli_si128(hi, 8)), m8)), d);
}
static float dot_lanes_avx2(const void* rowp, const float* x, const int n, const int dtype) {
    __m256 a0 = _mm256_setzero_ps(), a1 = _mm256_setzero_ps(), a2 = _mm256_setzero_ps(), a3 = _mm256_setzero_ps();
    int j = 0;
    if (dtype == XH_Q8_0 || dtype == XH_Q4_0) {  /* n % 32 == 0: one block per 32 columns */
        const uint8_t* row = (const uint8_t*)rowp;
        const size_t bs = xo_gq_bs(dtype);
        for (; j + 32 <= n; j += 32) {
            __m256 v[4];
            gq_block8(row + (size_t)(j / 32) * bs, dtype, v);
            a0 = _mm256_fmadd_ps(v[0], _mm256_loadu_ps(x + j), a0);
            a1 = _mm256_fmadd_ps(v[1], _mm256_loadu_ps(x + j + 8), a1);
            a2 = _mm256_fmadd_ps(v[2], _mm256_loadu_ps(x + j + 16), a2);
            a3 = _mm256_fmadd_ps(v[3], _mm256_loadu_ps(x + j + 24), a3);
        }
        return hsum8(a0, a1, a2, a3);
    }
    if (dtype == XH_F16) {
        const uint16_t* row = (const uint16_t*)rowp;
        for (; j + 32 <= n; j += 32) {
            a0 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(row + j))), _mm256_loadu_ps(x + j), a0);
            a1 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(row + j + 8))), _mm256_loadu_ps(x + j + 8), a1);
            a2 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(row + j + 16))), _mm256_loadu_ps(x + j + 16), a2);
            a3 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(row + j + 24))), _mm256_loadu_ps(x + j + 24), a3);
        }
        float val = hsum8(a0, a1, a2, a3);
        for (; j < n; j++) val += xo_f16_to_f32(row[j]) * x[j];
        return val;
    }
    const uint8_t* row = (const uint8_t*)rowp;
    const int e5 = dtype == XH_F8_E5M2;
    for (; j + 32 <= n; j += 32) {
        a0 = _mm256_fmadd_ps(f8x8(row + j, e5), _mm256_loadu_ps(x + j), a0);
        a1 = _mm256_fmadd_ps(f8x8(row + j + 8, e5), _mm256_loadu_ps(x + j + 8), a1);
        a2 = _mm256_fmadd_ps(f8x8(row + j + 16, e5), _mm256_loadu_ps(x + j + 16), a2);
        a3 = _mm256_fmadd_ps(f8x8(row + j + 24, e5), _mm256_loadu_ps(x + j + 24), a3);
    }
    float val = hsum8(a0, a1, a2, a3);
    for (; j < n; j++) val += (e5 ? f8e5m2_to_f32(row[j]) : f8e4m3_to_f32(row[j])) * x[j];
    return val;
}
#define XO_AVX512 __attribute__((target("avx512f,avx512bw,avx512vl,avx2,fma,f16c")))
XO_AVX512 static inline __m512 f8x16(const uint8_t* p, const int e5m2) {
    const __m512i b = _mm512_cvtepu8_epi32(_mm_loadu_si128((const __m128i*)p));
    const __m512i sg = _mm512_slli_epi32(_mm512_and_si512(b, _mm512_set1_epi32(0x80)), 24);
    const __m512i mg = _mm512_and_si512(b, _mm512_set1_epi32(0x7f));
    const __m512i u = _mm512_or_si512(sg, e5m2 ? _mm512_slli_epi32(mg, 21) : _mm512_slli_epi32(mg, 20));
    return _mm512_mul_ps(_mm512_castsi512_ps(u), _mm512_set1_ps(e5m2 ? 0x1p112f : 0x1p120f));
}
XO_AVX512 static float dot_lanes_avx512(const void* rowp, const float* x, const int n, const int dtype) {
    __m512 b0 = _mm512_setzero_ps(), b1 = _mm512_setzero_ps();  /* [a0 | a1], [a2 | a3] */
    int j = 0;
    if (dtype == XH_Q8_0 || dtype == XH_Q4_0) {
        const uint8_t* row = (const uint8_t*)rowp;
        const size_t bs = xo_gq_bs(dtype);
        for (; j + 32 <= n; j += 32) {
            __m256 v[4];
            gq_block8(row + (size_t)(j / 32) * bs, dtype, v);
            const __m512 v01 = _mm512_castpd_ps(_mm512_insertf64x4(_mm512_castpd256_pd512(_mm256_castps_pd(v[0])),
                                                                   _mm256_castps_pd(v[1]), 1));
            const __m512 v23 = _mm512_castpd_ps(_mm512_insertf64x4(_mm512_castpd256_pd512(_mm256_castps_pd(v[2])),
                                                                   _mm256_castps_pd(v[3]), 1));
            b0 = _mm512_fmadd_ps(v01, _mm512_loadu_ps(x + j), b0);
            b1 = _mm512_fmadd_ps(v23, _mm512_loadu_ps(x + j + 16), b1);
        }
        const __m256 h0 = _mm256_castpd_ps(_mm512_extractf64x4_pd(_mm512_castps_pd(b0), 1));
        const __m256 h1 = _mm256_castpd_ps(_mm512_extractf64x4_pd(_mm512_castps_pd(b1), 1));
        return hsum8(_mm512_castps512_ps256(b0), h0, _mm512_castps512_ps256(b1), h1);
    }
    if (dtype == XH_F16) {
        const uint16_t* row = (const uint16_t*)rowp;
        for (; j + 32 <= n; j += 32) {
            b0 = _mm512_fmadd_ps(_mm512_cvtph_ps(_mm256_loadu_si256((const __m256i*)(row + j))), _mm512_loadu_ps(x + j), b0);
            b1 = _mm512_fmadd_ps(_mm512_cvtph_ps(_mm256_loadu_si256((const __m256i*)(row + j + 16))), _mm512_loadu_ps(x + j + 16), b1);
        }
    } else {
        const uint8_t* row = (const uint8_t*)rowp;
        const int e5 = dtype == XH_F8_E5M2;
        for (; j + 32 <= n; j += 32) {
            b0 = _mm512_fmadd_ps(f8x16(row + j, e5), _mm512_loadu_ps(x + j), b0);
            b1 = _mm512_fmadd_ps(f8x16(row + j + 16, e5), _mm512_loadu_ps(x + j + 16), b1);
        }
    }
    /* upper halves through the AVX512F 64x4 extract (the 32x8 one is AVX512DQ) */
    const __m256 h0 = _mm256_castpd_ps(_mm512_extractf64x4_pd(_mm512_castps_pd(b0), 1));
    const __m256 h1 = _mm256_castpd_ps(_mm512_extractf64x4_pd(_mm512_castps_pd(b1), 1));
    float val = hsum8(_mm512_castps512_ps256(b0), h0, _mm512_castps512_ps256(b1), h1);
    if (dtype == XH_F16) {
        const uint16_t* row = (const uint16_t*)rowp;
        for (; j < n; j++) val += xo_f16_to_f32(row[j]) * x[j];
    } else {
        const uint8_t* row = (const uint8_t*)rowp;
        for (; j < n; j++) val += (dtype == XH_F8_E5M2 ? f8e5m2_to_f32(row[j]) : f8e4m3_to_f32(row[j])) * x[j];
    }
    return val;
}
typedef float (*xo_dot_fn)(const void*, const float*, int, int);
static xo_dot_fn dot_lanes = 0;
static int xo_isa_level = -1; /* 1 = AVX2/FMA/F16C, 2 = + AVX-512 */
static void pick_isa(void) {
    if (xo_isa_level >= 0) return;
    __builtin_cpu_init();
    const int avx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                       __builtin_cpu_supports("avx512vl") && !(getenv("XO_NO_AVX512") && atoi(getenv("XO_NO_AVX512")));
    dot_lanes = avx512 ? dot_lanes_avx512 : dot_lanes_avx2;
    xo_isa_level = avx512 ? 2 : 1;
}
int xo_isa(void) {
    pick_isa();
    return xo_isa_level;
}
#else
int xo_isa(void) { return 0; }
#endif

void xo_matmul(float* xout, const float* x, const void* w, const int dtype, const int n, const int d) {
    int i;
    if (scalar_order < 0) xo_matmul_order();
#ifdef XO_SIMD
    if ((dtype == XH_F16 || dtype == XH_F8_E4M3 || dtype == XH_F8_E5M2) && !scalar_order) {
        pick_isa();
        const size_t esz = dtype == XH_F16 ? 2 : 1;
#pragma omp parallel for schedule(static)
        for (i = 0; i < d; i++) xout[i] = dot_lanes((const char*)w + (size_t)i * n * esz, x, n, dtype);
        return;
    }
    if (xo_gq(dtype) && !scalar_order && n % 32 == 0) {
        /* gguf blocks dequantized 32 at a time (exact), then the lanes order of the f32 loop */
        pick_isa();
        const size_t rb = (size_t)n / 32 * xo_gq_bs(dtype);
#pragma omp parallel for schedule(static)
        for (i = 0; i < d; i++) xout[i] = dot_lanes((const char*)w + (size_t)i * rb, x, n, dtype);
        return;
    }
#endif
#ifdef XO_SIMD
    if (dtype == XH_F16) {
        /* sequential order: the same left-to-right product + sum as the generic loop below
         * (separate multiply and add), with the f16 -> f32 conversions done 8 at a time */
        const uint16_t* W = (const uint16_t*)w;
#pragma omp parallel for schedule(static)
        for (i = 0; i < d; i++) {
            const uint16_t* row = W + (size_t)i * n;
            float val = 0.0f, f[8];
            int j = 0;
            for (; j + 8 <= n; j += 8) {
                _mm256_storeu_ps(f, _mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(row + j))));
                for (int e = 0; e < 8; e++) {
                    const float p = f[e] * x[j + e];
                    val += p;
                }
            }
            for (; j < n; j++) val += xo_f16_to_f32(row[j]) * x[j];
            xout[i] = val;
        }
        return;
    }
#endif
#define XO_MATMUL_LOOP(T, DEC)                                              \
    {                                                                       \
        const T* W = (const T*)w;                                           \
        _Pragma("omp parallel for schedule(static)")                        \
        for (i = 0; i < d; i++) {                                           \
            const T* row = W + (size_t)i * n;                               \
            float val = 0.0f;                                               \
            for (int j = 0; j < n; j++) val += DEC(row[j]) * x[j];          \
            xout[i] = val;                                                  \
        }                                                                   \
    }
#define DEC_F32(v) (v)
    switch (dtype) {
        case XH_F32: XO_MATMUL_LOOP(float, DEC_F32); break;
        case XH_F16: XO_MATMUL_LOOP(uint16_t, xo_f16_to_f32); break;
        case XH_BF16: XO_MATMUL_LOOP(uint16_t, bf16_to_f32); break;
        case XH_F8_E4M3: XO_MATMUL_LOOP(uint8_t, f8e4m3_to_f32); break;
        case XH_F8_E5M2: XO_MATMUL_LOOP(uint8_t, f8e5m2_to_f32); break;
        case XH_Q8: XO_MATMUL_LOOP(int8_t, q8_to_f32); break;
        case XH_Q8_0: case XH_Q4_0: {
            /* dequantize (quants.py) then the reference's row loop */
            const size_t nb = (size_t)n / 32, bs = xo_gq_bs(dtype);
#pragma omp parallel for schedule(static)
            for (i = 0; i < d; i++) {
                const uint8_t* row = (const uint8_t*)w + (size_t)i * nb * bs;
                float val = 0.0f, f[32];
                for (size_t b = 0; b < nb; b++) {  /* one block's 32 values, then the same sums in j order */
                    const uint8_t* blk = row + b * bs;
                    for (int k = 0; k < 32; k++) f[k] = xo_gq_elem(dtype, blk, k);
                    const float* xb = x + b * 32;
                    for (int k = 0; k < 32; k++) val += f[k] * xb[k];
                }
                xout[i] = val;
            }
            break;
        }
        default: for (i = 0; i < d; i++) xout[i] = NAN; break;
    }
#undef XO_MATMUL_LOOP
#undef DEC_F32
}

/* rmsnorm, src/infer.cpp:224-236 (dispatch :238-251): serial sum of squares in index
 * order; o = x * (1/sqrtf(ss/n + eps)) * w.  Safe in place (o == x), as :628. */
void xo_rmsnorm(float* o, const float* x, const void* w, const int dtype, const int size, const float eps) {
    float rms = 0.0f;
    for (int i = 0; i < size; ++i) rms += x[i] * x[i];
    rms = sqrtf(rms / (float)size + eps);
    const float scale = 1.0f / rms;
    for (int i = 0; i < size; ++i) {
        const float wi = dtype == XH_BF16 ? bf16_to_f32(((const uint16_t*)w)[i]) : ((const float*)w)[i];
        o[i] = x[i] * scale * wi;
    }
}

/* softmax, src/infer.cpp:280-297 */
static void softmax(float* o, const float* x, const int size) {
    float score_max = -FLT_MAX; /* std::numeric_limits<float>::lowest() */
    for (int i = 0; i < size; ++i)
        if (x[i] > score_max) score_max = x[i];
    float score_sum = 0.0f;
    for (int i = 0; i < size; ++i) {
        o[i] = expf(x[i] - score_max);
        score_sum += o[i];
    }
    for (int i = 0; i < size; ++i) o[i] /= score_sum;
}

/* gelu / silu / clip, src/infer.cpp:299-303 */
static inline float gelu(const float x) { return 0.5f * x * (1.0f + tanhf(0.797885f * (x + 0.044715f * x * x * x))); }
static inline float silu(const float x) { return x / (1.0f + expf(-x)); }
static inline float clip(const float x, const float v) { return x < -v ? -v : (x > v ? v : x); }

/* rope, src/infer.cpp:305-322: adjacent pairs (i, i+1) rotated by pos * theta^(-j/rot). */
void xo_rope(float* vec, const int d, const int head_dim, const int pos, const float theta, const int rotary_dim) {
    for (int i = 0; i < d; i += 2) {
        const int j_head = i % head_dim;
        const float freq = j_head >= rotary_dim ? 0.f : 1.0f / powf(theta, (float)j_head / (float)rotary_dim);
        const float val = (float)pos * freq;
        const float fcr = cosf(val);
        const float fci = sinf(val);
        const float v0 = vec[i];
        const float v1 = vec[i + 1];
        vec[i] = v0 * fcr - v1 * fci;
        vec[i + 1] = v0 * fci + v1 * fcr;
    }
}

/* f16 -> f32 in the attention loops: F16C's conversion is exact and equal to xo_f16_to_f32 for
 * every non-NaN code (a NaN stays a NaN, its payload may differ) */
#ifdef XO_SIMD
static inline float f16f(const uint16_t h) { return _cvtsh_ss(h); }
#else
static inline float f16f(const uint16_t h) { return xo_f16_to_f32(h); }
#endif

/* attn, src/infer.cpp:325-359: one head over kv_len ring slots in slot order. */
static void attn(float* xout, float* atth, const float* qh, const uint16_t* kh, const uint16_t* vh,
                 const int head_dim, const int n_kv_heads, const int kv_len) {
    const int kv_stride = n_kv_heads * head_dim;
    const float sqrt_head_dim = 1.0f / sqrtf((float)head_dim);
    for (int t = 0; t < kv_len; ++t) {
        float score = 0.0f;
        for (int i = 0; i < head_dim; ++i) score += qh[i] * f16f(kh[(size_t)t * kv_stride + i]);
        atth[t] = score * sqrt_head_dim;
    }
    softmax(atth, atth, kv_len);
    /* xout[i] = sum over t in slot order of atth[t] * v[t][i] (src/infer.cpp:349-356), with the
     * loops interchanged so V is read row by row: every xout[i] still receives its terms in slot
     * order, so the sums are the same bits as the column-major loop (which re-walks the whole
     * ring once per dimension: ~100x slower at 32k slots) */
    float vacc[512];
    for (int i = 0; i < head_dim; ++i) vacc[i] = 0.0f;
    for (int t = 0; t < kv_len; ++t) {
        const uint16_t* vr = vh + (size_t)t * kv_stride;
        const float a = atth[t];
        for (int i = 0; i < head_dim; ++i) vacc[i] += a * f16f(vr[i]);
    }
    for (int i = 0; i < head_dim; ++i) xout[i] = vacc[i];
}

/* mha_cpu, src/infer.cpp:498-517 */
void xo_mha(float* xout, float* att, const uint16_t* kb, const uint16_t* vb, const float* q, const int head_dim,
            const int kv_len, const int max_seq_len, const int n_heads, const int n_kv_heads) {
    const int q_per_kv_head = n_heads / n_kv_heads;
    int h;
#pragma omp parallel for schedule(static)
    for (h = 0; h < n_heads; h++) {
        const int kv_head_offset = (h / q_per_kv_head) * head_dim;
        attn(xout + head_dim * h, att + (size_t)max_seq_len * h, q + head_dim * h, kb + kv_head_offset,
             vb + kv_head_offset, head_dim, n_kv_heads, kv_len);
    }
}

/* Sampler::sample_argmax, src/sampler.cpp:19-30 (max starts at FLT_MIN; first max wins) */
int xo_sample_argmax(const float* logits, const int vocab) {
    int argmax = 0;
    float max_val = FLT_MIN;
    for (int i = 0; i < vocab; ++i)
        if (logits[i] > max_val) { max_val = logits[i]; argmax = i; }
    return argmax;
}

/* Sampler::sample_prob, src/sampler.cpp:3-17 */
float xo_sample_prob(const float* logits, const int vocab, const int index) {
    float max_val = FLT_MIN;
    for (int i = 0; i < vocab; ++i)
        if (logits[i] > max_val) max_val = logits[i];
    float sum = 0;
    for (int i = 0; i < vocab; ++i) sum += expf(logits[i] - max_val);
    return expf(logits[index] - max_val) / sum;
}

int xo_num_threads(void) { return omp_get_max_threads(); }
void xo_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

/* ------------------------------------------------------------------------------------ */
/* model + InferenceState, src/model.h:96-284, src/model.cpp                             */
/* ------------------------------------------------------------------------------------ */
typedef struct { int dtype; const void* data; } xo_tensor;

typedef struct {
    xo_tensor t[XH_NUM_KINDS];
    uint16_t* key_cache;   /* float16_t[max_seq_len * kv_dim], src/model.cpp:102-103 */
    uint16_t* value_cache;
} xo_block;

struct xo_model {
    xh_config c;
    xo_tensor embed, final_norm, wcls;
    xo_block* blocks;
    /* InferenceState, src/model.h:97-108 */
    float *x, *xb, *xb2, *hb, *hb2, *q, *k, *v, *att, *logits;
    /* the same state in double for the fp64 evaluation (xo_set_precision(m, 1)), allocated on
     * first use */
    double *dx, *dxb, *dxb2, *dhb, *dhb2, *dq, *dk, *dv, *datt;
    int prec64;
};

static void* xcalloc(size_t n, size_t sz) { return calloc(n ? n : 1, sz); }

xo_model* xo_create(const xh_config* cfg) {
    if (cfg->head_dim <= 0 || cfg->head_dim > 512) return NULL; /* attn's row accumulators hold 512 */
    xo_model* m = (xo_model*)xcalloc(1, sizeof(xo_model));
    if (!m) return NULL;
    m->c = *cfg;
    const xh_config* c = cfg;
    const size_t q_dim = (size_t)c->n_heads * c->head_dim, kv_dim = (size_t)c->n_kv_heads * c->head_dim;
    m->blocks = (xo_block*)xcalloc((size_t)c->n_layers, sizeof(xo_block));
    for (int l = 0; l < c->n_layers; l++) {
        m->blocks[l].key_cache = (uint16_t*)xcalloc((size_t)c->max_seq_len * kv_dim, 2);
        m->blocks[l].value_cache = (uint16_t*)xcalloc((size_t)c->max_seq_len * kv_dim, 2);
    }
    /* xb2 sized max(dim, q_dim): the reference sizes it [dim] and writes q_dim floats */
    const size_t xb2n = q_dim > (size_t)c->dim ? q_dim : (size_t)c->dim;
    m->x = (float*)xcalloc(c->dim, 4);
    m->xb = (float*)xcalloc(c->dim, 4);
    m->xb2 = (float*)xcalloc(xb2n, 4);
    /* hb also receives the Wo output [dim] (src/infer.cpp:447); size it for both */
    const size_t hbn = (size_t)c->hidden_dim > (size_t)c->dim ? (size_t)c->hidden_dim : (size_t)c->dim;
    m->hb = (float*)xcalloc(hbn, 4);
    m->hb2 = (float*)xcalloc(c->hidden_dim, 4);
    m->q = (float*)xcalloc(q_dim, 4);
    m->k = (float*)xcalloc(kv_dim, 4);
    m->v = (float*)xcalloc(kv_dim, 4);
    m->att = (float*)xcalloc((size_t)c->n_heads * c->max_seq_len, 4);
    m->logits = (float*)xcalloc(c->vocab_size, 4);
    return m;
}

void xo_destroy(xo_model* m) {
    if (!m) return;
    for (int l = 0; l < m->c.n_layers; l++) {
        free(m->blocks[l].key_cache);
        free(m->blocks[l].value_cache);
    }
    free(m->blocks);
    free(m->x); free(m->xb); free(m->xb2); free(m->hb); free(m->hb2);
    free(m->q); free(m->k); free(m->v); free(m->att); free(m->logits);
    free(m->dx); free(m->dxb); free(m->dxb2); free(m->dhb); free(m->dhb2);
    free(m->dq); free(m->dk); free(m->dv); free(m->datt);
    free(m);
}

void xo_reset(xo_model* m) {
    const size_t kv_dim = (size_t)m->c.n_kv_heads * m->c.head_dim;
    for (int l = 0; l < m->c.n_layers; l++) {
        memset(m->blocks[l].key_cache, 0, (size_t)m->c.max_seq_len * kv_dim * 2);
        memset(m->blocks[l].value_cache, 0, (size_t)m->c.max_seq_len * kv_dim * 2);
    }
}

int xo_set_tensor(xo_model* m, int kind, int layer, int dtype, const void* data) {
    if (kind < 0 || kind >= XH_NUM_KINDS || !data) return XH_E_INVALID;
    xo_tensor t = {dtype, data};
    if (kind == XH_EMBED) m->embed = t;
    else if (kind == XH_FINAL_NORM) m->final_norm = t;
    else if (kind == XH_WCLS) m->wcls = t;
    else {
        if (layer < 0 || layer >= m->c.n_layers) return XH_E_INVALID;
        m->blocks[layer].t[kind] = t;
    }
    return 0;
}

const float* xo_logits(const xo_model* m) { return m->logits; }
uint16_t* xo_key_cache(xo_model* m, int layer) { return m->blocks[layer].key_cache; }
uint16_t* xo_value_cache(xo_model* m, int layer) { return m->blocks[layer].value_cache; }

/* bytes of one [n]-element row (gguf blocks: n/32 blocks) */
static size_t row_bytes(int dtype, size_t n) { return xo_gq(dtype) ? n / 32 * xo_gq_bs(dtype) : n * dtype_bits(dtype) / 8; }

/* Model::active_bytes, src/model.cpp:12-35 */
size_t xo_active_bytes(const xo_model* m, size_t pos) {
    const xh_config* c = &m->c;
    size_t bytes = 0;
    const size_t q_dim = (size_t)c->n_heads * c->head_dim, kv_dim = (size_t)c->n_kv_heads * c->head_dim;
    bytes += row_bytes(m->embed.dtype, c->dim);
    bytes += row_bytes(m->final_norm.dtype, c->dim);
    bytes += (size_t)c->vocab_size * row_bytes(m->wcls.dtype, c->dim);
    for (int l = 0; l < c->n_layers; ++l) {
        const xo_tensor* t = m->blocks[l].t;
        bytes += row_bytes(t[XH_ATTN_NORM].dtype, c->dim);
        bytes += row_bytes(t[XH_FFN_NORM].dtype, c->dim);
        bytes += q_dim * row_bytes(t[XH_WQ].dtype, c->dim);
        bytes += kv_dim * row_bytes(t[XH_WK].dtype, c->dim);
        bytes += kv_dim * row_bytes(t[XH_WV].dtype, c->dim);
        bytes += (size_t)c->dim * row_bytes(t[XH_WO].dtype, q_dim);
        bytes += (size_t)c->hidden_dim * row_bytes(t[XH_W1].dtype, c->dim);
        bytes += (size_t)c->dim * row_bytes(t[XH_W2].dtype, c->hidden_dim);
        bytes += (size_t)c->hidden_dim * row_bytes(t[XH_W3].dtype, c->dim);
        const size_t kv_len = (size_t)c->max_seq_len < pos + 1 ? (size_t)c->max_seq_len : pos + 1;
        bytes += 2 * kv_len * c->n_kv_heads * c->head_dim * 2;
    }
    return bytes;
}

/* Model::_copy_embedding, src/infer.cpp:553-602 */
static void copy_embedding(xo_model* m, const int token) {
    for (int i = 0; i < m->c.dim; ++i) m->x[i] = xo_decode_row(m->embed.dtype, m->embed.data, (size_t)token, m->c.dim, i);
}

/* Block::_block_cpu, src/infer.cpp:365-496 */
static void block_cpu(xo_model* m, const xo_block* b, const int pos, const int kv_sink, const int kv_pos,
                      const int kv_len) {
    const xh_config* c = &m->c;
    const xo_tensor* t = b->t;
    /* attention pre-norm :374-382 */
    xo_rmsnorm(m->xb, m->x, t[XH_ATTN_NORM].data, t[XH_ATTN_NORM].dtype, c->dim, c->norm_eps);
    const int q_dim = c->n_heads * c->head_dim;
    const int kv_dim = c->n_kv_heads * c->head_dim;
    /* qkv matmuls :388-390 */
    xo_matmul(m->q, m->xb, t[XH_WQ].data, t[XH_WQ].dtype, c->dim, q_dim);
    xo_matmul(m->k, m->xb, t[XH_WK].data, t[XH_WK].dtype, c->dim, kv_dim);
    xo_matmul(m->v, m->xb, t[XH_WV].data, t[XH_WV].dtype, c->dim, kv_dim);
    /* qkv clip :392-399 */
    for (int i = 0; i < q_dim; ++i) m->q[i] = clip(m->q[i], c->qkv_clip);
    for (int i = 0; i < kv_dim; ++i) {
        m->k[i] = clip(m->k[i], c->qkv_clip);
        m->v[i] = clip(m->v[i], c->qkv_clip);
    }
    uint16_t* kb = b->key_cache;
    uint16_t* vb = b->value_cache;
    /* RoPE :407-408 */
    xo_rope(m->q, q_dim, c->head_dim, pos, c->rope_theta, c->rotary_dim);
    xo_rope(m->k, kv_dim, c->head_dim, pos, c->rope_theta, c->rotary_dim);
    /* kv cache write (fp32 -> fp16) :411-414 */
    for (int i = 0; i < kv_dim; ++i) {
        kb[(size_t)kv_pos * kv_dim + i] = xo_f32_to_f16(m->k[i]);
        vb[(size_t)kv_pos * kv_dim + i] = xo_f32_to_f16(m->v[i]);
    }
    /* sink re-rotation by +1 position, fp16 round trip :421-431 */
    for (int r = 0; r < kv_sink; r++) {
        for (int i = 0; i < kv_dim; ++i) m->k[i] = xo_f16_to_f32(kb[(size_t)r * kv_dim + i]);
        xo_rope(m->k, kv_dim, c->head_dim, 1, c->rope_theta, c->rotary_dim);
        for (int i = 0; i < kv_dim; i++) kb[(size_t)r * kv_dim + i] = xo_f32_to_f16(m->k[i]);
    }
    /* multi-head attention :435-444 */
    xo_mha(m->xb2, m->att, kb, vb, m->q, c->head_dim, kv_len, c->max_seq_len, c->n_heads, c->n_kv_heads);
    /* output projection + residual :447-452 */
    xo_matmul(m->hb, m->xb2, t[XH_WO].data, t[XH_WO].dtype, q_dim, c->dim);
    for (int i = 0; i < c->dim; ++i) m->x[i] += m->hb[i];
    /* ffn pre-norm :455-463 */
    xo_rmsnorm(m->xb, m->x, t[XH_FFN_NORM].data, t[XH_FFN_NORM].dtype, c->dim, c->norm_eps);
    /* GLU ffn :468-494 */
    xo_matmul(m->hb, m->xb, t[XH_W1].data, t[XH_W1].dtype, c->dim, c->hidden_dim);
    xo_matmul(m->hb2, m->xb, t[XH_W3].data, t[XH_W3].dtype, c->dim, c->hidden_dim);
    if (c->act == XH_ACT_GELU) {
        for (int i = 0; i < c->hidden_dim; ++i) m->hb[i] = gelu(m->hb[i]) * m->hb2[i];
    } else {
        for (int i = 0; i < c->hidden_dim; ++i) m->hb[i] = silu(m->hb[i]) * m->hb2[i];
    }
    xo_matmul(m->xb2, m->hb, t[XH_W2].data, t[XH_W2].dtype, c->hidden_dim, c->dim);
    for (int i = 0; i < c->dim; ++i) m->x[i] += m->xb2[i];
}

/* ------------------------------------------------------------------------------------ */
/* fp64 evaluation of the same algorithm (xo_set_precision(m, 1))                           */
/* ------------------------------------------------------------------------------------ */
/* Every product, sum, norm, softmax, activation and residual of src/infer.cpp:224-638 in
 * double, so the result is the reference algorithm's value up to ~1e-16 relative: a
 * precision-independent yardstick for "how far is an f32 evaluation from the algorithm's
 * exact value".  Kept exactly as the reference defines them, because they are part of the
 * algorithm rather than of its arithmetic precision: the weights (decoded to their exact
 * values), the fp16 K/V cache (every stored K/V element rounded to fp16, src/infer.cpp:410-414,
 * and the sink re-rotation's fp16 round trip :421-431), the rope angle table (the float
 * expressions `1.0f / powf(theta, j / rot)` and `pos * freq` of :310-314; cos / sin of that angle
 * in double) and the FLT_MIN start of the sampler.  Logits are returned rounded to float. */
void xo_set_precision(xo_model* m, int p) { m->prec64 = p != 0; }
int xo_precision(const xo_model* m) { return m->prec64; }

static double* dcalloc(size_t n) { return (double*)xcalloc(n, sizeof(double)); }

static int alloc64(xo_model* m) {
    if (m->dx) return 0;
    const xh_config* c = &m->c;
    const size_t q_dim = (size_t)c->n_heads * c->head_dim, kv_dim = (size_t)c->n_kv_heads * c->head_dim;
    const size_t xb2n = q_dim > (size_t)c->dim ? q_dim : (size_t)c->dim;
    const size_t hbn = (size_t)c->hidden_dim > (size_t)c->dim ? (size_t)c->hidden_dim : (size_t)c->dim;
    m->dx = dcalloc(c->dim); m->dxb = dcalloc(c->dim); m->dxb2 = dcalloc(xb2n);
    m->dhb = dcalloc(hbn); m->dhb2 = dcalloc(c->hidden_dim);
    m->dq = dcalloc(q_dim); m->dk = dcalloc(kv_dim); m->dv = dcalloc(kv_dim);
    m->datt = dcalloc((size_t)c->n_heads * c->max_seq_len);
    return m->dx && m->dxb && m->dxb2 && m->dhb && m->dhb2 && m->dq && m->dk && m->dv && m->datt ? 0 : XH_E_INVALID;
}

/* matmul (src/infer.cpp:104-135) with double products and a double accumulator */
static void matmul64(double* xout, const double* x, const void* w, const int dtype, const int n, const int d) {
    int i;
    if (dtype == XH_F16) {
        const uint16_t* W = (const uint16_t*)w;
#pragma omp parallel for schedule(static)
        for (i = 0; i < d; i++) {
            const uint16_t* row = W + (size_t)i * n;
            int j = 0;
            double val = 0.0;
#ifdef XO_SIMD
            __m256d a0 = _mm256_setzero_pd(), a1 = _mm256_setzero_pd();
            for (; j + 8 <= n; j += 8) {
                const __m256 f = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(row + j)));
                a0 = _mm256_fmadd_pd(_mm256_cvtps_pd(_mm256_castps256_ps128(f)), _mm256_loadu_pd(x + j), a0);
                a1 = _mm256_fmadd_pd(_mm256_cvtps_pd(_mm256_extractf128_ps(f, 1)), _mm256_loadu_pd(x + j + 4), a1);
            }
            double t[4];
            _mm256_storeu_pd(t, _mm256_add_pd(a0, a1));
            val = (t[0] + t[1]) + (t[2] + t[3]);
#endif
            for (; j < n; j++) val += (double)xo_f16_to_f32(row[j]) * x[j];
            xout[i] = val;
        }
        return;
    }
    if (dtype == XH_F8_E4M3 || dtype == XH_F8_E5M2 || dtype == XH_Q8) {
        /* one-byte codes: the decode of each of the 256 codes, looked up */
        double tab[256];
        for (int c = 0; c < 256; c++) {
            const uint8_t b = (uint8_t)c;
            tab[c] = xo_decode(dtype, &b, 0);
        }
        const uint8_t* W = (const uint8_t*)w;
#pragma omp parallel for schedule(static)
        for (i = 0; i < d; i++) {
            const uint8_t* row = W + (size_t)i * n;
            double v0 = 0.0, v1 = 0.0;
            int j = 0;
            for (; j + 2 <= n; j += 2) {
                v0 += tab[row[j]] * x[j];
                v1 += tab[row[j + 1]] * x[j + 1];
            }
            for (; j < n; j++) v0 += tab[row[j]] * x[j];
            xout[i] = v0 + v1;
        }
        return;
    }
    if (dtype == XH_BF16) {
        const uint16_t* W = (const uint16_t*)w;
#pragma omp parallel for schedule(static)
        for (i = 0; i < d; i++) {
            const uint16_t* row = W + (size_t)i * n;
            double val = 0.0;
            for (int j = 0; j < n; j++) val += (double)bf16_to_f32(row[j]) * x[j];
            xout[i] = val;
        }
        return;
    }
    if (xo_gq(dtype)) {
        /* gguf blocks: each block's 32 values decoded once, then the same sums in j order */
        const size_t nb = (size_t)n / 32, bs = xo_gq_bs(dtype);
#pragma omp parallel for schedule(static)
        for (i = 0; i < d; i++) {
            const uint8_t* row = (const uint8_t*)w + (size_t)i * nb * bs;
            double val = 0.0;
            float f[32];
            for (size_t b = 0; b < nb; b++) {
                for (int k = 0; k < 32; k++) f[k] = xo_gq_elem(dtype, row + b * bs, k);
                for (int k = 0; k < 32; k++) val += (double)f[k] * x[b * 32 + k];
            }
            xout[i] = val;
        }
        return;
    }
#pragma omp parallel for schedule(static)
    for (i = 0; i < d; i++) {
        double val = 0.0;
        for (int j = 0; j < n; j++) val += (double)xo_decode_row(dtype, w, (size_t)i, (size_t)n, (size_t)j) * x[j];
        xout[i] = val;
    }
}

/* rmsnorm, src/infer.cpp:224-236 */
static void rmsnorm64(double* o, const double* x, const void* w, const int dtype, const int size, const float eps) {
    double ss = 0.0;
    for (int i = 0; i < size; ++i) ss += x[i] * x[i];
    const double scale = 1.0 / sqrt(ss / (double)size + (double)eps);
    for (int i = 0; i < size; ++i) {
        const double wi = dtype == XH_BF16 ? bf16_to_f32(((const uint16_t*)w)[i]) : ((const float*)w)[i];
        o[i] = x[i] * scale * wi;
    }
}

/* rope, src/infer.cpp:305-322: the reference's float angle, rotated in double */
static void rope64(double* vec, const int d, const int head_dim, const int pos, const float theta, const int rotary_dim) {
    for (int i = 0; i < d; i += 2) {
        const int j_head = i % head_dim;
        const float freq = j_head >= rotary_dim ? 0.f : 1.0f / powf(theta, (float)j_head / (float)rotary_dim);
        const float val = (float)pos * freq;
        const double fcr = cos((double)val), fci = sin((double)val);
        const double v0 = vec[i], v1 = vec[i + 1];
        vec[i] = v0 * fcr - v1 * fci;
        vec[i + 1] = v0 * fci + v1 * fcr;
    }
}

/* attn + softmax, src/infer.cpp:280-297, 325-359 */
static void attn64(double* xout, double* atth, const double* qh, const uint16_t* kh, const uint16_t* vh,
                   const int head_dim, const int n_kv_heads, const int kv_len) {
    const int kv_stride = n_kv_heads * head_dim;
    const double inv_sqrt = 1.0 / sqrt((double)head_dim);
    double mx = -DBL_MAX;
    for (int t = 0; t < kv_len; ++t) {
        double score = 0.0;
        for (int i = 0; i < head_dim; ++i) score += qh[i] * (double)f16f(kh[(size_t)t * kv_stride + i]);
        atth[t] = score * inv_sqrt;
        if (atth[t] > mx) mx = atth[t];
    }
    double sum = 0.0;
    for (int t = 0; t < kv_len; ++t) {
        atth[t] = exp(atth[t] - mx);
        sum += atth[t];
    }
    for (int t = 0; t < kv_len; ++t) atth[t] /= sum;
    double vacc[512];  /* row-major V walk, each sum in slot order (as attn) */
    for (int i = 0; i < head_dim; ++i) vacc[i] = 0.0;
    for (int t = 0; t < kv_len; ++t) {
        const uint16_t* vr = vh + (size_t)t * kv_stride;
        const double a = atth[t];
        for (int i = 0; i < head_dim; ++i) vacc[i] += a * (double)f16f(vr[i]);
    }
    for (int i = 0; i < head_dim; ++i) xout[i] = vacc[i];
}

static inline double clip64(const double x, const double v) { return x < -v ? -v : (x > v ? v : x); }
/* the fp16 cache store of a double: rounded once to float, then to fp16 as the reference */
static inline uint16_t f16_of(const double v) { return xo_f32_to_f16((float)v); }

/* Block::_block_cpu, src/infer.cpp:365-496, in double */
static void block64(xo_model* m, const xo_block* b, const int pos, const int kv_sink, const int kv_pos,
                    const int kv_len) {
    const xh_config* c = &m->c;
    const xo_tensor* t = b->t;
    const int q_dim = c->n_heads * c->head_dim, kv_dim = c->n_kv_heads * c->head_dim;
    const double vclip = (double)c->qkv_clip;
    rmsnorm64(m->dxb, m->dx, t[XH_ATTN_NORM].data, t[XH_ATTN_NORM].dtype, c->dim, c->norm_eps);
    matmul64(m->dq, m->dxb, t[XH_WQ].data, t[XH_WQ].dtype, c->dim, q_dim);
    matmul64(m->dk, m->dxb, t[XH_WK].data, t[XH_WK].dtype, c->dim, kv_dim);
    matmul64(m->dv, m->dxb, t[XH_WV].data, t[XH_WV].dtype, c->dim, kv_dim);
    for (int i = 0; i < q_dim; ++i) m->dq[i] = clip64(m->dq[i], vclip);
    for (int i = 0; i < kv_dim; ++i) {
        m->dk[i] = clip64(m->dk[i], vclip);
        m->dv[i] = clip64(m->dv[i], vclip);
    }
    uint16_t* kb = b->key_cache;
    uint16_t* vb = b->value_cache;
    rope64(m->dq, q_dim, c->head_dim, pos, c->rope_theta, c->rotary_dim);
    rope64(m->dk, kv_dim, c->head_dim, pos, c->rope_theta, c->rotary_dim);
    for (int i = 0; i < kv_dim; ++i) {
        kb[(size_t)kv_pos * kv_dim + i] = f16_of(m->dk[i]);
        vb[(size_t)kv_pos * kv_dim + i] = f16_of(m->dv[i]);
    }
    for (int r = 0; r < kv_sink; r++) {
        for (int i = 0; i < kv_dim; ++i) m->dk[i] = xo_f16_to_f32(kb[(size_t)r * kv_dim + i]);
        rope64(m->dk, kv_dim, c->head_dim, 1, c->rope_theta, c->rotary_dim);
        for (int i = 0; i < kv_dim; i++) kb[(size_t)r * kv_dim + i] = f16_of(m->dk[i]);
    }
    const int qpk = c->n_heads / c->n_kv_heads;
    int h;
#pragma omp parallel for schedule(static)
    for (h = 0; h < c->n_heads; h++) {
        const int kvo = (h / qpk) * c->head_dim;
        attn64(m->dxb2 + (size_t)c->head_dim * h, m->datt + (size_t)c->max_seq_len * h, m->dq + (size_t)c->head_dim * h,
               kb + kvo, vb + kvo, c->head_dim, c->n_kv_heads, kv_len);
    }
    matmul64(m->dhb, m->dxb2, t[XH_WO].data, t[XH_WO].dtype, q_dim, c->dim);
    for (int i = 0; i < c->dim; ++i) m->dx[i] += m->dhb[i];
    rmsnorm64(m->dxb, m->dx, t[XH_FFN_NORM].data, t[XH_FFN_NORM].dtype, c->dim, c->norm_eps);
    matmul64(m->dhb, m->dxb, t[XH_W1].data, t[XH_W1].dtype, c->dim, c->hidden_dim);
    matmul64(m->dhb2, m->dxb, t[XH_W3].data, t[XH_W3].dtype, c->dim, c->hidden_dim);
    for (int i = 0; i < c->hidden_dim; ++i) {
        const double g = m->dhb[i];
        const double a = c->act == XH_ACT_GELU ? 0.5 * g * (1.0 + tanh(0.797885 * (g + 0.044715 * g * g * g)))
                                               : g / (1.0 + exp(-g));
        m->dhb[i] = a * m->dhb2[i];
    }
    matmul64(m->dxb2, m->dhb, t[XH_W2].data, t[XH_W2].dtype, c->hidden_dim, c->dim);
    for (int i = 0; i < c->dim; ++i) m->dx[i] += m->dxb2[i];
}

static int forward64(xo_model* m, const int token, const int pos, const int mode, const int kv_sink, const int kv_pos,
                     const int kv_len) {
    const xh_config* c = &m->c;
    if (alloc64(m)) return XH_E_INVALID;
    for (int i = 0; i < c->dim; ++i) m->dx[i] = xo_decode_row(m->embed.dtype, m->embed.data, (size_t)token, c->dim, i);
    for (int l = 0; l < c->n_layers; l++) block64(m, &m->blocks[l], pos, kv_sink, kv_pos, kv_len);
    if (mode == XH_HYDRATE_KV_CACHE) return 0;
    rmsnorm64(m->dx, m->dx, m->final_norm.data, m->final_norm.dtype, c->dim, c->norm_eps);
    /* lm_head into dhb-sized scratch is too small for the vocabulary: rows in chunks */
    double out[256];
    for (int r0 = 0; r0 < c->vocab_size; r0 += 256) {
        const int rows = c->vocab_size - r0 < 256 ? c->vocab_size - r0 : 256;
        const size_t rb = row_bytes(m->wcls.dtype, c->dim);
        matmul64(out, m->dx, (const char*)m->wcls.data + (size_t)r0 * rb, m->wcls.dtype, c->dim, rows);
        for (int i = 0; i < rows; i++) m->logits[r0 + i] = (float)out[i];
    }
    return 0;
}

/* Model::_forward_cpu, src/infer.cpp:604-638 */
int xo_forward(xo_model* m, const int token, const int pos, const int mode) {
    const xh_config* c = &m->c;
    if (token < 0 || token >= c->vocab_size || pos < 0) return XH_E_INVALID;
    if (!m->embed.data || !m->final_norm.data || !m->wcls.data) return XH_E_STATE;
    for (int l = 0; l < c->n_layers; l++)
        for (int k = XH_ATTN_NORM; k <= XH_W3; k++)
            if (!m->blocks[l].t[k].data) return XH_E_STATE;
    /* ring / sink bookkeeping :611-613 */
    const int kv_sink = pos >= c->max_seq_len ? KV_SINKS : 0;
    const int kv_pos = kv_sink + (pos - kv_sink) % (c->max_seq_len - kv_sink);
    const int kv_len = pos >= c->max_seq_len ? c->max_seq_len : pos + 1;
    if (m->prec64) return forward64(m, token, pos, mode, kv_sink, kv_pos, kv_len);
    copy_embedding(m, token);
    for (int l = 0; l < c->n_layers; l++) block_cpu(m, &m->blocks[l], pos, kv_sink, kv_pos, kv_len);
    if (mode == XH_HYDRATE_KV_CACHE) return 0; /* :620-623 */
    xo_rmsnorm(m->x, m->x, m->final_norm.data, m->final_norm.dtype, c->dim, c->norm_eps); /* :626-634 */
    xo_matmul(m->logits, m->x, m->wcls.data, m->wcls.dtype, c->dim, c->vocab_size);       /* :637 */
    return 0;
}
