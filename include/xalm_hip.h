/*
 * xalm_hip.h — C ABI of the MI355X (gfx950) single-batch decode path.
 *
 * This is the drop-in boundary for Xalm's per-token forward pass.  The reference C++ API it
 * replaces (all paths under jubruckne/Xalm @ 2025-03-21):
 *
 *   void Model::forward(const InferenceState& s, int token, int pos,
 *                       InferenceMode mode = OUTPUT_LOGITS) const;      src/model.h:272
 *     -> Model::_forward_cpu                                             src/infer.cpp:604-638
 *     -> Block::block / _block_cpu                                       src/model.cpp:37-46,
 *                                                                        src/infer.cpp:365-496
 *   struct InferenceState { x, xb, xb2, hb, hb2, q, k, v, att, logits }  src/model.h:96-156
 *   Model::from_xalm (host Tensor buffers, per-layer KV caches)          src/model.cpp:48-118
 *   enum class Device { CPU }  (the `-d` switch)                         src/model.h:21-23
 *   Exposed-for-tests ops: attn / mha_cpu / mha_cuda / matmul            src/model.h:286-316
 *
 * Conventions: plain pointers and sizes only; every call returns 0 on success or a
 * nonzero XH_E* code; xh_last_error() gives a message.  One host thread per context; a
 * context is one live sequence (as the reference Model: KV and scratch are shared).
 * Weights are COPIED into device memory by xh_upload (the caller keeps ownership).
 */
#ifndef XALM_HIP_H
#define XALM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- element types: the reference `Type` ids (src/types.h:505-514) ------------------ */
enum xh_dtype {
    XH_F32 = 1,
    XH_F16 = 2,
    XH_BF16 = 3,
    XH_F8_E4M3 = 6,
    XH_F8_E5M2 = 7,
    XH_U8 = 8,
    XH_Q8 = 9, /* int8 * 0.01f, src/types.h:423-424 */
    /* The converter's gguf blocks (convert.py:176-187 `--type q8_0 / q4_0`, quants.py): 32
     * elements per block, an f16 scale d first.  Q8_0 (quants.py:441-463): 34 B = d + 32
     * int8, value d*q.  Q4_0 (quants.py:281-311): 18 B = d + 16 bytes, byte j holding element
     * j (low nibble) and j+16 (high nibble), value d*(nibble-8).  Tensors are uploaded in that
     * file layout ([rows][cols/32 blocks], header shape = bytes per row); the reference C++
     * runtime cannot parse them (src/types.h:468-499), so the ids are this build's. */
    XH_Q8_0 = 20,
    XH_Q4_0 = 21
};

/* ---- tensor kinds (names as in .xalm, src/model.cpp:83-114) ------------------------ */
enum xh_tensor_kind {
    XH_EMBED = 0,      /* embed.weight          [vocab, dim]              */
    XH_ATTN_NORM = 1,  /* l.N.attn.norm.weight  [dim]                     */
    XH_FFN_NORM = 2,   /* l.N.mlp.norm.weight   [dim]                     */
    XH_WQ = 3,         /* l.N.attn.q.weight     [n_heads*head_dim, dim]   */
    XH_WK = 4,         /* l.N.attn.k.weight     [n_kv_heads*head_dim, dim]*/
    XH_WV = 5,         /* l.N.attn.v.weight     [n_kv_heads*head_dim, dim]*/
    XH_WO = 6,         /* l.N.attn.down.weight  [dim, n_heads*head_dim]   */
    XH_W1 = 7,         /* l.N.mlp.gate.weight   [hidden_dim, dim]         */
    XH_W2 = 8,         /* l.N.mlp.down.weight   [dim, hidden_dim]         */
    XH_W3 = 9,         /* l.N.mlp.up.weight     [hidden_dim, dim]         */
    XH_FINAL_NORM = 10,/* output.norm.weight    [dim]                     */
    XH_WCLS = 11,      /* output.weight (or embed.weight if tied) [vocab, dim] */
    XH_NUM_KINDS = 12
};

/* InferenceMode, src/model.h:249-252 */
enum xh_mode { XH_HYDRATE_KV_CACHE = 0, XH_OUTPUT_LOGITS = 1 };
/* ActivationType, src/model.h:12-15 */
enum xh_act { XH_ACT_GELU = 0, XH_ACT_SILU = 1 };

enum xh_status {
    XH_OK = 0,
    XH_E_INVALID = 1,   /* bad argument / shape / dtype mismatch (reference: throw invalid_argument) */
    XH_E_HIP = 2,       /* HIP runtime error */
    XH_E_STATE = 3,     /* call out of order, e.g. forward before all weights uploaded */
    XH_E_NOMEM = 4
};

/* POD mirror of `Config` (src/model.h:25-91); max_seq_len already resolved (cap 4096 or -T). */
typedef struct xh_config {
    int32_t dim;
    int32_t hidden_dim;
    int32_t head_dim;
    int32_t n_layers;
    int32_t n_heads;
    int32_t n_kv_heads;
    int32_t vocab_size;
    int32_t max_seq_len;
    float rope_theta;
    int32_t rotary_dim;
    float norm_eps;
    int32_t act;            /* enum xh_act */
    float qkv_clip;         /* FLT_MAX when absent (src/model.h:84-85) */
    int32_t tie_word_embeddings;
} xh_config;

typedef struct xh_ctx xh_ctx;

/* Create a device context on HIP device `device_ordinal`: allocates the fp16 KV rings
 * (2 * n_layers * max_seq_len * n_kv_heads*head_dim) and the device InferenceState. */
int xh_create(const xh_config* cfg, int device_ordinal, xh_ctx** out);
void xh_destroy(xh_ctx* ctx);
const char* xh_last_error(const xh_ctx* ctx); /* ctx may be NULL: last create error */

/* Copy one host tensor (`bytes` must equal shape*elem size) to the device.  `layer` is
 * ignored for embed/final_norm/wcls.  Shape and dtype are validated against the config
 * (mirrors the load_tensor checks, src/model.cpp:62-81).  Matrices of one layer that
 * the kernels fuse (q/k/v, gate/up) must share one dtype. */
int xh_upload(xh_ctx* ctx, int tensor_kind, int layer, int dtype, const void* host, size_t bytes);

/* The same upload read straight from a file: `bytes` at absolute `offset` of `path` (a
 * .xalm tensor, convert.py:248-321; the reference reads it into a host Tensor first,
 * src/xalm.h:90-192, src/model.cpp:48-118).  The range is memory-mapped, pinned for the
 * copy and moved by one DMA; no host copy of the tensor is made.  Same validation as
 * xh_upload, plus the range must lie inside the file.  Synchronous. */
int xh_upload_file(xh_ctx* ctx, int tensor_kind, int layer, int dtype, const char* path, uint64_t offset,
                   size_t bytes);

/* Benchmark weights without a checkpoint: fill the tensor slot on the device with the
 * deterministic values of include/xalm_synth.h (element i of the logical [rows][cols]
 * tensor = xs_value(seed, i, mean, std) rounded to `dtype`).  The CPU baseline builds the
 * bit-identical host copy from the same header.  Q8 is not supported. */
int xh_upload_synthetic(xh_ctx* ctx, int tensor_kind, int layer, int dtype, uint64_t seed, float mean, float std);
/* Fill KV ring rows [slot0, slot0+n_slots) of one layer with synthetic fp16 N(0, std)-like values. */
int xh_kv_fill_synthetic(xh_ctx* ctx, int layer, int which, int slot0, int n_slots, uint64_t seed, float std);

/* One token of Model::forward (src/model.cpp:120-122 / src/infer.cpp:604-638).
 * kv_sink/kv_pos/kv_len follow src/infer.cpp:611-613.  logits_out: caller-owned host
 * float[vocab] (may be NULL; required for nothing).  Synchronous. */
int xh_forward(xh_ctx* ctx, int token, int pos, int mode, float* logits_out);

/* Greedy decode fully on device: starting from the current logits (left by the last
 * OUTPUT_LOGITS forward at position pos-1), repeat n_steps times:
 *   tok = argmax(logits) (Sampler::sample_argmax semantics, src/sampler.cpp:19-30);
 *   tokens_out[i] = tok; forward(tok, pos + i, OUTPUT_LOGITS).
 * No host round trip per token (one graph replay per step).  If stop_token_a/b >= 0 the
 * host stops after the step that produced one of them; returns the count in *n_done. */
int xh_decode_greedy(xh_ctx* ctx, int pos, int n_steps, int stop_token_a, int stop_token_b,
                     int* tokens_out, int* n_done);

/* Hydrate: forward tokens[0..n) at positions pos0.. (HYDRATE_KV_CACHE for all but the last,
 * which computes logits if want_logits), the prompt loop of run_completion
 * (src/main.cpp:94-100) in one call.  logits_out may be NULL. */
int xh_prefill(xh_ctx* ctx, const int* tokens, int n, int pos0, int want_logits, float* logits_out);

/* Perplexity scoring, the loop of run_perplexity (src/main.cpp:243-254) in one call: forward
 * tokens[0..n-1) at positions pos0.. with logits and write probs_out[i] =
 * Sampler::sample_prob(tokens[i+1]) (src/sampler.cpp:3-17; n-1 floats, caller-owned).  The
 * logits stay on the device; with XH_OPT_PREFILL on, each pass computes every token's logits
 * with one lm_head GEMM.  n >= 2.  The caller takes log and sums, as the
 * reference does in double. */
int xh_perplexity(xh_ctx* ctx, const int* tokens, int n, int pos0, float* probs_out);

/* Debug timelines (device clock, 100 MHz; each launch overwrites).  enable bits: 2 = every
 * attention + Wo launch writes [workgroup][8] stamps (start, attention done / hand-off passed,
 * end, split known, scores done, p.V done, partial drained); 8 = every W1/W3 launch writes
 * [workgroup][4] (start, x staged, end, XCD << 32 | HW_ID); 16 = the last layer's launches and the
 * lm_head write [workgroup][4 | 8] into their own regions (tools/layer_trace.py); 0 = off,
 * -1 = unchanged.  Copies min(cap, *len) words of the trace buffer to `out` first. */
int xh_debug_trace(xh_ctx* ctx, int enable, uint64_t* out, int cap, int* len);

/* Copy the current device logits to the host. */
int xh_get_logits(xh_ctx* ctx, float* logits_out);

/* Zero the KV rings and state (a fresh sequence). */
int xh_reset(xh_ctx* ctx);

/* Direct KV ring access, for tests and for pre-filling long contexts.
 * which: 0 = key cache, 1 = value cache.  Rows are [slot][n_kv_heads*head_dim] fp16 bits. */
int xh_kv_write(xh_ctx* ctx, int layer, int which, int slot0, int n_slots, const uint16_t* host);
int xh_kv_read(xh_ctx* ctx, int layer, int which, int slot0, int n_slots, uint16_t* host);

/* Bytes the forward pass reads per token: Model::active_bytes(pos), src/model.cpp:12-35. */
size_t xh_active_bytes(const xh_ctx* ctx, size_t pos);

/* Graph capture of the per-token step (default on).  Off = eager launches (debugging). */
int xh_set_graphs(xh_ctx* ctx, int enable);

/* Launch-structure variants.  XH_OPT_FUSE_ATTN_WO (default 1): 1 = attention and Wo (+ residual)
 * in one launch with an in-launch hand-off (attn_wo.h); 0 = two launches.  Same math. */
/* XH_OPT_PREFILL (default 1): xh_prefill / xh_perplexity process the prompt in passes, each
 * weight matrix streamed once per pass into a GEMM.  1 = f16 and fp8 weights on the LDS-tiled MFMA
 * GEMM (gemm16.h) in passes of up to PF_TOK_MM = 2048 tokens (fp8 matrices through their exact f16 image),
 * activations as exact f16 hi + lo pairs under a power-of-two row scale (|x - (hi + lo) / s| <=
 * 2^-22 |x|, a 22-bit mantissa where the reference's f32 has 24), products exact, f32
 * accumulation in an order fixed by the tiling (the same bits on every run); other weight dtypes
 * on the f32-input MFMA kernel (activations exactly as the reference) in passes of 64 tokens;
 * 2 = the split-f16 register-streaming MFMA kernel wherever the weights convert exactly to f16
 * (f16, fp8), passes of 64 tokens; 3 = f32-input MFMA only; 4 = as 1 with vendor hipBLASLt in place
 * of gemm16.h (passes of 512 tokens, the heuristic's first algorithm: deterministic per library
 * build); 0 = one forward per token (the reference's loop, src/main.cpp:94-100).  Same math per
 * token up to f32 rounding. */
/* XH_OPT_PREFILL_GLU_SPLIT (default 1): where the W2 GEMM takes split-f16 input, the GLU
 * epilogue of the W1/W3 GEMM writes those f16 hi/lo halves directly (one launch), and each
 * residual add runs in one launch with the following rmsnorm split; 0 = GLU to f32 first, then
 * split in the W2 GEMM's input pass, and residual and rmsnorm as separate launches.
 * Bit-identical results; a debug knob so tests cover both routes. */
/* XH_OPT_PREFILL_ATTN (default 1): the batched path's causal attention on MFMA tiles (32 query
 * rows x 32-slot K/V tiles per wave, running max/sum, q and p as exact f16 hi + lo pairs), the
 * K/V tiles shared by the 4 waves of a workgroup through an LDS ring (head_dim 128); 2 = the same
 * arithmetic with every wave reading its own tiles (bit-identical to 1); 0 = one workgroup per
 * token and KV head, split-KV (the decode attention's blocks).
 * Option id 4 (XH_OPT_COL_KV_MAX, removed in round 3 with the column-form attention) is no
 * longer accepted: xh_set_option / xh_get_option return XH_E_INVALID for it. */
/* XH_OPT_PREFILL_ATTN_SPLIT (default 1): under XH_OPT_PREFILL_ATTN 1, a pass too short to fill the
 * chip with (KV head, 128-row query tile) workgroups walks a long history in splits (each with its
 * own running max / sum), merged per row in split order afterwards (deterministic); 0 = one
 * workgroup walks the whole history.  Same math up to f32 rounding. */
enum xh_option {
    XH_OPT_FUSE_ATTN_WO = 1,
    XH_OPT_PREFILL = 2,
    XH_OPT_PREFILL_GLU_SPLIT = 3,
    XH_OPT_PREFILL_ATTN = 5,
    XH_OPT_PREFILL_ATTN_SPLIT = 6
};
int xh_set_option(xh_ctx* ctx, int option, int value);
int xh_get_option(const xh_ctx* ctx, int option, int* value);

/* ---- exposed-for-tests ops (src/model.h:286-316), host pointers in/out -------------- */
/* matmul: xout[d] = W[d,n] @ x[n], W of `dtype` (src/infer.cpp:185-216). */
int xh_op_matmul(float* xout, const float* x, const void* w, int dtype, int n, int d);
/* rmsnorm (src/infer.cpp:224-251), weight of dtype F32 or BF16. */
int xh_op_rmsnorm(float* o, const float* x, const void* weight, int dtype, int size, float eps);
/* rope in place on vec[d] (src/infer.cpp:305-322). */
int xh_op_rope(float* vec, int d, int head_dim, int pos, float theta, int rotary_dim);
/* mha_cuda (src/model.h:308-313): xout[n_heads*head_dim]; kb/vb fp16 [max_seq_len][n_kv_heads*head_dim]. */
int xh_op_mha(float* xout, const uint16_t* kb, const uint16_t* vb, const float* q, int head_dim,
              int kv_len, int max_seq_len, int n_heads, int n_kv_heads);

/* The prompt-pass GEMM of XH_OPT_PREFILL 1 (gemm16.h): y[t][r] = sum_k w[r][k] * (xh[t][k] + xl[t][k])
 * with f16 w [rows][K], f16 xh / xl [n][K] and f32 y [n][rows] (the K slices' partials summed in
 * slice order, as the prompt path's epilogue).  K % 64 == 0; ks = K slices (0: the prompt path's
 * choice for this shape).  No reference counterpart: the matmul of src/infer.cpp:104-135 over n
 * tokens at once. */
int xh_op_prompt_gemm(float* y, const uint16_t* w, const uint16_t* xh, const uint16_t* xl, int rows, int K, int n,
                      int ks);

/* ---- timing hooks used by bench.py (HIP events on the context's own stream) -------- */
/* Average device time (microseconds) of one launch of kernel `which` (0 = the fused
 * gate/up matvec, 1 = qkv, 2 = wo, 3 = down, 4 = lm_head, 5 = attention) over `iters`
 * back-to-back launches with the current step parameters (layers rotate, so the Infinity Cache
 * never serves a repeat). */
int xh_time_kernel(xh_ctx* ctx, int which, int iters, float* avg_us);
/* Bytes one launch of that kernel must move (algorithmic). */
size_t xh_kernel_bytes(const xh_ctx* ctx, int which, int kv_len);

#ifdef __cplusplus
}
#endif
#endif /* XALM_HIP_H */
