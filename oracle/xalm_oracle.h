/*
 * xalm_oracle.h — CPU oracle: a C restatement of the reference forward path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (libxalm_hip.so, libxalm_host.so, bin/xalm) never links it.
 *
 * Restates jubruckne/Xalm src/infer.cpp (the reference cannot be compiled on x86: it
 * needs <arm_neon.h> and C++23 <format>/<print>).  Parity pinning: the
 * forward is checked against HuggingFace transformers logits on .xalm fixtures written by
 * the reference's own convert.py (tests/golden/, tests/test_oracle.py).
 */
#ifndef XALM_ORACLE_H
#define XALM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/xalm_hip.h" /* shared POD config + dtype / tensor-kind enums */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct xo_model xo_model;

xo_model* xo_create(const xh_config* cfg);
void xo_destroy(xo_model* m);
/* Borrow (no copy) one weight tensor; layer ignored for embed/final_norm/wcls. */
int xo_set_tensor(xo_model* m, int kind, int layer, int dtype, const void* data);
/* Model::_forward_cpu (src/infer.cpp:604-638). Returns 0 on success. */
int xo_forward(xo_model* m, int token, int pos, int mode);
const float* xo_logits(const xo_model* m);
/* 1: evaluate this model's forward in double (products, sums, norms, softmax, activations,
 * residuals) with the fp16 K/V cache and the reference's float rope angles kept; logits
 * rounded to float.  0 (default): the reference's f32 arithmetic. */
void xo_set_precision(xo_model* m, int p);
int xo_precision(const xo_model* m);
uint16_t* xo_key_cache(xo_model* m, int layer);   /* fp16 bits [max_seq_len][kv_dim] */
uint16_t* xo_value_cache(xo_model* m, int layer);
size_t xo_active_bytes(const xo_model* m, size_t pos);
void xo_reset(xo_model* m);

/* ops (exposed for tests in the reference, src/model.h:286-316) */
void xo_matmul(float* xout, const float* x, const void* w, int dtype, int n, int d);
/* f16 / fp8 in-row summation order: 0 = 8-wide FMA lanes (default), 1 = sequential */
void xo_set_matmul_order(int order);
int xo_matmul_order(void);
/* the lanes order's instruction set, picked at run time: 2 = AVX-512, 1 = AVX2, 0 = scalar */
int xo_isa(void);
void xo_rmsnorm(float* o, const float* x, const void* w, int dtype, int size, float eps);
void xo_rope(float* vec, int d, int head_dim, int pos, float theta, int rotary_dim);
void xo_mha(float* xout, float* att, const uint16_t* kb, const uint16_t* vb, const float* q,
            int head_dim, int kv_len, int max_seq_len, int n_heads, int n_kv_heads);
float xo_decode(int dtype, const void* data, size_t idx);
/* element i of row `row` of a [rows][n] tensor (gguf blocks: the converter's block layout) */
float xo_decode_row(int dtype, const void* data, size_t row, size_t n, size_t i);
/* quantize n_blocks blocks of 32 floats into gguf Q8_0 / Q4_0 block bytes (xalm_synth.h) */
void xo_quantize_gq(int dtype, const float* v, size_t n_blocks, uint8_t* out);
uint16_t xo_f32_to_f16(float f);
float xo_f16_to_f32(uint16_t h);
int xo_sample_argmax(const float* logits, int vocab);
float xo_sample_prob(const float* logits, int vocab, int index);
int xo_num_threads(void);
/* OpenMP threads for the following calls (the 1-thread CPU baseline) */
void xo_set_threads(int n);
void xo_fill_synthetic(void* dst, size_t rows, size_t cols, int dtype, uint64_t seed, float mean, float std);

#ifdef __cplusplus
}
#endif
#endif
