// standalone.h — single-op kernels (test ops and the graph engine's embedding gather).
// Included by xalm_hip.hip only: non-template kernels must live in one translation unit.
#pragma once

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
__global__ void embed_kernel(const void* emb, int dtype, int dim, float* x, const StepParams* sp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < dim) x[i] = dec1(dtype, emb, (size_t)sp->token * dim + i);
}

}  // namespace xalm
