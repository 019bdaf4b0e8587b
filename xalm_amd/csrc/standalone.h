// standalone.h — single-op kernels (test ops and the graph engine's embedding gather).
// Included by xalm_hip.hip only: non-template kernels must live in one translation unit.
#pragma once

#include <float.h>

#include "gemv.h"

namespace xalm {

// rmsnorm as a standalone op (xh_op_rmsnorm), same reduction as the fused prologue.
__global__ __launch_bounds__(256) void rmsnorm_kernel(float* o, const float* x, const void* w, int dtype, int n,
                                                       float eps) {
    __shared__ float red[4];
    const float scale = block_rms_scale<256>(x, n, eps, red);
    for (int i = threadIdx.x; i < (n >> 2); i += 256) {
        const float4 v = ((const float4*)x)[i];
        const float4 wv = load_norm4(w, dtype, i);
        ((float4*)o)[i] = make_float4(v.x * scale * wv.x, v.y * scale * wv.y, v.z * scale * wv.z, v.w * scale * wv.w);
    }
}

// rope as a standalone op (xh_op_rope), same device function as the QKV epilogue.
__global__ void rope_kernel(float* vec, int d, int head_dim, int pos, const float* freq) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * p >= d) return;
    float v0 = vec[2 * p], v1 = vec[2 * p + 1];
    rope_pair(v0, v1, 2 * p, head_dim, pos, freq);
    vec[2 * p] = v0;
    vec[2 * p + 1] = v1;
}

// Model::_copy_embedding (src/infer.cpp:553-602): x = dec(embed[token, :])
__global__ void embed_kernel(const void* emb, int dtype, int dim, float* x, const StepParams* sp,
                             const float* rope_freq, float* rope_cs, int half) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < dim) x[i] = dec_row(dtype, emb, (size_t)sp->token, dim, i);
    if (blockIdx.x == 0) rope_table(rope_cs, rope_freq, half, sp->pos, threadIdx.x);
}

// Greedy decode step head: argmax over the lm_head workgroups' candidates (Sampler::
// sample_argmax, src/sampler.cpp:19-30: the first maximum among logits > FLT_MIN, else token
// 0), the decode-loop bookkeeping of argmax_advance (tokens[step], step, token, positions,
// src/infer.cpp:611-613) and x = embed[token] (Model::_copy_embedding,
// src/infer.cpp:553-602), in one 1024-thread workgroup.
constexpr int ARGMAX_CANDS = 1024;
__global__ __launch_bounds__(1024) void argmax_embed_kernel(const unsigned long long* cand, StepParams* sp,
                                                            int* tokens, int cap, const void* emb, int dtype,
                                                            int dim, float* x, const float* rope_freq,
                                                            float* rope_cs, int half) {
    __shared__ unsigned long long kb[16];
    __shared__ int tok_s, pos_s;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned long long best = cand[tid];  // ARGMAX_CANDS == blockDim.x
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o, 64);
        best = other > best ? other : best;
    }
    if (lane == 0) kb[wid] = best;
    __syncthreads();
    if (tid == 0) {
        unsigned long long bb = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) bb = kb[w] > bb ? kb[w] : bb;
        const int tok = argmax_key_index(bb);
        if (sp->step < cap) tokens[sp->step] = tok;
        sp->step += 1;
        sp->token = tok;
        step_positions(sp, sp->pos_next);
        sp->pos_next += 1;
        tok_s = tok;
        pos_s = sp->pos;
    }
    __syncthreads();
    rope_table(rope_cs, rope_freq, half, pos_s, tid);
    for (int i = tid; i < dim; i += 1024) x[i] = dec_row(dtype, emb, (size_t)tok_s, dim, i);
}

// Candidates from logits already on the device (the first greedy step after logits that no
// EPI_LOGITS launch produced): cand[0] = best key, the rest 0.
__global__ __launch_bounds__(1024) void logits_cand_kernel(const float* logits, int vocab, unsigned long long* cand) {
    __shared__ unsigned long long kb[16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned long long best = 0;
    for (int i = tid; i < vocab; i += 1024) {
        const float v = logits[i];
        if (v > FLT_MIN) {
            const unsigned long long k = argmax_key(v, i);
            best = k > best ? k : best;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o, 64);
        best = other > best ? other : best;
    }
    if (lane == 0) kb[wid] = best;
    __syncthreads();
    unsigned long long bb = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) bb = kb[w] > bb ? kb[w] : bb;
    cand[tid] = tid == 0 ? bb : 0ull;
}

// Sampler::sample_prob (src/sampler.cpp:3-17) of one logits row per workgroup: max over the
// row starting at FLT_MIN (the reference's quirk: a row of logits all below it is shifted by
// FLT_MIN, not by its own max), then expf(l[target] - max) / sum_i expf(l[i] - max).  The sum
// is a tree, not the reference's index-ordered loop: float rounding differs, nothing else.
// Row t: logits + t * stride; probs[t] = the probability of targets[t].
__global__ __launch_bounds__(1024) void token_prob_kernel(const float* logits, int vocab, size_t stride,
                                                          const int* targets, float* probs) {
    __shared__ float red[16];
    const float* l = logits + (size_t)blockIdx.x * stride;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    float m = FLT_MIN;
    for (int i = tid; i < vocab; i += 1024) m = l[i] > m ? l[i] : m;  // NaN never wins, as `>`
    m = wave_max(m);
    if (lane == 0) red[wid] = m;
    __syncthreads();
    m = red[0];
#pragma unroll
    for (int w = 1; w < 16; w++) m = red[w] > m ? red[w] : m;
    __syncthreads();
    float s = 0.f;
    for (int i = tid; i < vocab; i += 1024) s += expf(l[i] - m);
    s = wave_sum(s);
    if (lane == 0) red[wid] = s;
    __syncthreads();
    if (tid == 0) {
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < 16; w++) tot += red[w];
        probs[blockIdx.x] = expf(l[targets[blockIdx.x]] - m) / tot;
    }
}

}  // namespace xalm
