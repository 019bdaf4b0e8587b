// prefill.h — batched prompt processing: the prompt loop of run_completion
// (jubruckne/Xalm src/main.cpp:94-100, HYDRATE_KV_CACHE src/infer.cpp:620-623) for up to
// PF_TOK tokens per pass, so every weight matrix is streamed once per pass instead of once
// per token.  Same math per token as the decode path (src/infer.cpp:365-496); the matrix
// products run on the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 products, f32
// accumulation — a k-ordered fmaf chain, MI355X_MICROARCH.md "Matrix cores"), so activations
// stay f32 exactly as in the reference; only the summation order differs.
//
// GEMM layout: Y[t][r] = sum_k X[t][k] W[r][k], W row-major [rows][K] as uploaded.  One wave
// owns 32 rows x one K slice x up to 64 tokens (two 32x32 f32 accumulator tiles).  Lane l
// streams 16 bytes of row r0 + (l & 31) at k = kb + E (l >> 5) and decodes them to E floats:
// they are the B operand of E MFMAs whose A operand is X[t][same k] (MFMA 32x32x2 f32 operand
// map: A[i = l & 31][k = l >> 5], B[k = l >> 5][j = l & 31]), so weights go HBM -> VGPR ->
// MFMA with no LDS staging; X (a few MB) is read from L2.  K slices write f32 partials
// [slice][t][r]; a second kernel sums them in slice order and applies the decode path's
// epilogue (clip + rope + fp16 K/V write, silu * up, residual add).
#pragma once

#include "attention.h"
#include "gemv.h"

namespace xalm {

constexpr int PF_TOK = 64;       // tokens per pass (two MFMA token tiles)
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

template <int DT>
__global__ __launch_bounds__(PF_THREADS) void prefill_gemm_kernel(const PfGemmArgs a) {
    constexpr int E = WDec<DT>::E;
    constexpr int ESZ = 16 / E;  // bytes per element
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * PF_WAVES + (threadIdx.x >> 6);
    const int n_rt = (a.rows + 31) / 32;
    if (gw >= n_rt * a.ks) return;
    const int rt = gw / a.ks, s = gw - rt * a.ks;
    const int j = lane & 31, h = lane >> 5;
    const int r = rt * 32 + j;
    const int kslice = a.K / a.ks;
    const int k0 = s * kslice, k1 = k0 + kslice;
    const char* wrow = (const char*)a.w + (size_t)min(r, a.rows - 1) * a.row_bytes;
    const int n_tt = (a.n + 31) / 32;
    // token rows of this lane's A operand in each tile (clamped: rows past n are not stored)
    const float* x0 = a.x + (size_t)min(j, a.n - 1) * a.K;
    const float* x1 = a.x + (size_t)min(32 + j, a.n - 1) * a.K;
    f32x16 acc0 = {}, acc1 = {};
    for (int kb = k0; kb < k1; kb += 2 * E) {
        const int k = kb + E * h;
        const u32x4 wv = *(const u32x4*)(wrow + (size_t)k * ESZ);
        float wf[E];
        WDec<DT>::dec(wv, wf);
        float xa[E];
#pragma unroll
        for (int q = 0; q < E / 4; q++) {
            const float4 v = *(const float4*)(x0 + k + 4 * q);
            xa[4 * q] = v.x; xa[4 * q + 1] = v.y; xa[4 * q + 2] = v.z; xa[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int e = 0; e < E; e++) acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[e], wf[e], acc0, 0, 0, 0);
        if (n_tt > 1) {
#pragma unroll
            for (int q = 0; q < E / 4; q++) {
                const float4 v = *(const float4*)(x1 + k + 4 * q);
                xa[4 * q] = v.x; xa[4 * q + 1] = v.y; xa[4 * q + 2] = v.z; xa[4 * q + 3] = v.w;
            }
#pragma unroll
            for (int e = 0; e < E; e++) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[e], wf[e], acc1, 0, 0, 0);
        }
    }
    if (r >= a.rows) return;
    // D map: column j = lane & 31 (row r), row i = (reg & 3) + 8 (reg >> 2) + 4 h (token)
    float* out = a.part + (size_t)s * a.n * a.rows + r;
#pragma unroll
    for (int reg = 0; reg < 16; reg++) {
        const int t = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (t < a.n) out[(size_t)t * a.rows] = acc0[reg];
        if (n_tt > 1 && 32 + t < a.n) out[(size_t)(32 + t) * a.rows] = acc1[reg];
    }
}

// Per-pass token scalars
struct PfEpiArgs {
    const float* part;  // [ks][n][rows]
    int ks, n, rows;
    int epi;            // EPI_QKV / EPI_RESID / EPI_GLU / EPI_STORE
    float* out;         // RESID: X [n][rows] (+=); GLU: H [n][rows/2]; STORE: [n][rows]
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
    // one thread per output pair (rows are even for QKV / GLU; RESID / STORE take both)
    const int pairs = a.rows / 2;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.n * pairs) return;
    const int t = idx / pairs, r = 2 * (idx - t * pairs);
    float v0 = 0.f, v1 = 0.f;
    for (int s = 0; s < a.ks; s++) {  // slice order: fixed
        const float* p = a.part + ((size_t)s * a.n + t) * a.rows + r;
        v0 += p[0];
        v1 += p[1];
    }
    if (a.epi == EPI_RESID) {
        float* o = a.out + (size_t)t * a.rows + r;
        o[0] += v0;
        o[1] += v1;
    } else if (a.epi == EPI_STORE) {
        float* o = a.out + (size_t)t * a.rows + r;
        o[0] = v0;
        o[1] = v1;
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
    const size_t base = (size_t)tokens[blockIdx.x] * dim;
    for (int i = threadIdx.x; i < dim; i += 256) x[(size_t)blockIdx.x * dim + i] = dec1(dtype, emb, base + i);
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

}  // namespace xalm
