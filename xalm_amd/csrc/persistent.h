// persistent.h — one-launch decode engine: every phase of every token inside one kernel.
//
// Same math as the multi-launch path (gemv.h, attention.h), reorganised for MI355X:
// * grid = one 1024-thread workgroup per CU, all co-resident; workgroup b owns a fixed slice
//   of the rows of every matrix (and the matching rows of the residual stream x);
// * phases per layer: QKV -> attention -> Wo -> W1/W3 -> W2, then lm_head (+ argmax) per
//   token; a phase's output is published with write-through (sc1) stores, every storing wave
//   drains vmcnt, one lane adds to the phase counter; consumers poll that counter (one lane,
//   relaxed, bounded) and read the data with sc1 loads: the fence-free hand-off form of
//   MI355X_MICROARCH.md "Valid forms" row 1;
// * the weight stream does not depend on activations, so each wave requests the first
//   chunk of its next phase's rows BEFORE it waits on the hand-off: HBM keeps streaming
//   across every dependency (no launch boundaries, no ramp / tail per matrix);
// * the argmax of the logits is reduced per workgroup during lm_head and merged by every
//   workgroup from 256 candidates, so the next token needs no extra hand-off, and the
//   embedding row is read directly as layer 0's input.
// Every spin is bounded (s_memrealtime, 2 s); on timeout the kernel sets an error word and
// every workgroup drains out.
#pragma once

#include <float.h>

#include "attention.h"
#include "gemv.h"

namespace xalm {

constexpr int PK_THREADS = 512;
constexpr int PK_WAVES = PK_THREADS / 64;
constexpr int PK_ROWS = 2;
constexpr int PK_U = 8;
constexpr int PK_PHASES = 5;  // per layer: qkv, att, wo, w13, w2

struct PkLayer {
    const void* wqkv;
    const void* wo;
    const void* w13;
    const void* w2;
    const void* attn_norm;
    const void* ffn_norm;
    uint16_t* kc;
    uint16_t* vc;
};

struct PkArgs {
    // model
    int n_layers, dim, hidden, q_dim, kv_dim, head_dim, n_heads, n_kv_heads, vocab, max_seq_len;
    float eps, qkv_clip;
    int act, norm_dt;           // norm weights dtype (F32 / BF16), same for every norm
    const void* embed;
    int embed_dt;
    const void* final_norm;
    const void* wcls;
    const PkLayer* layers;
    const float* rope_freq;
    const float* sink_cos;
    const float* sink_sin;
    // state
    float* x;        // [dim] residual stream
    float* q;        // [q_dim]
    float* attn;     // [q_dim] attention output
    float* hb;       // [hidden]
    float* logits;   // [vocab]
    float* part_o;   // [nsplit][n_heads][hd]
    float* part_ml;  // [nsplit][n_heads][2]
    unsigned long long* cand;  // [gridDim.x] per-workgroup argmax candidate
    int nsplit;
    // sync
    unsigned* counters;  // [n_layers * PK_PHASES + 1], zeroed before every launch
    int* tickets;        // [n_kv_heads], zero between launches
    int* err;            // timeout flag
    // work of this launch
    const int* prompt;   // tokens fed (device), n_prompt of them
    int n_prompt;
    int n_gen;           // greedy tokens generated after the prompt
    int pos0;            // position of the first token of this launch
    int logits_last;     // compute logits for the last token
    int stop_a, stop_b;  // greedy stop tokens (-1: none)
    int* tokens_out;     // generated tokens
    int* n_done;         // generated count (written by workgroup 0)
    // debug timeline (null: off): for the last token of the launch, workgroups 0, nblk/2 and
    // nblk-1 store s_memrealtime at [wg][l][phase][0 = hand-off passed, 1 = published]
    unsigned long long* trace;
};
constexpr int PK_TRACE_WG = 3;
__host__ __device__ constexpr int pk_trace_len(int n_layers) { return (n_layers + 1) * PK_PHASES * 2 + 2; }

// threadIdx.x behind an empty asm: thread-derived addresses are recomputed where they are
// used instead of being hoisted out of the token/layer loops and kept live (they spilled)
__device__ __forceinline__ int pk_tid() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
// the kernel's argument block, re-read (scalar loads) in every phase for the same reason
__device__ __forceinline__ const struct PkArgs* pk_args() {
    const PkArgs* p = (const PkArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

__device__ __forceinline__ uint64_t pk_now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ unsigned long long pk_key(const float v, const int idx) { return argmax_key(v, idx); }

// Counters are addressed logically (a.counters + k) and stored sharded: counter k occupies
// PK_SHARDS lines of its own, one per XCD, so 256 arrivals are 8 parallel fan-ins of 32
// (MI355X_MICROARCH.md "fanin": ~11-13 ns per serialized atomic).
constexpr int PK_SHARDS = 8;
constexpr int PK_SHARD_STRIDE = 32;  // uints: one 128-B line per shard
constexpr int PK_CSLOT = PK_SHARDS * PK_SHARD_STRIDE;
__device__ __forceinline__ unsigned* pk_shard(const unsigned* c, const int shard) {
    unsigned* base = pk_args()->counters;
    return base + (size_t)(c - base) * PK_CSLOT + shard * PK_SHARD_STRIDE;
}
__device__ __forceinline__ int pk_xcc() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 3)" : "=s"(v));
    return v & (PK_SHARDS - 1);
}

// publish: every wave's sc1 stores drained, then one add (after a workgroup barrier) on this
// XCD's shard
__device__ __forceinline__ void pk_signal(unsigned* c, const unsigned add = 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (pk_tid() == 0)
        __hip_atomic_fetch_add(pk_shard(c, pk_xcc()), add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned pk_count(const unsigned* c) {
    unsigned s = 0;
#pragma unroll
    for (int k = 0; k < PK_SHARDS; k++) s += __hip_atomic_load(pk_shard(c, k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return s;
}

// wait until *c >= target (one lane polls, relaxed, with s_sleep; 2 s bound); false on error
__device__ __forceinline__ bool pk_wait(const unsigned* c, const unsigned target, int* err, int* lds_flag) {
    if (pk_tid() == 0) {
        int ok = 1;
        const uint64_t t0 = pk_now();
        unsigned spins = 0;
        while (pk_count(c) < target) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 255) == 0) {
                if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { ok = 0; break; }
                if (pk_now() - t0 > 200000000ull) {  // 2 s at 100 MHz
                    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
            }
        }
        *lds_flag = ok;
    }
    __syncthreads();
    const int ok = *lds_flag;
    __syncthreads();
    return ok != 0;
}

// x image for a gemv phase: src (sc1) optionally rms-normalised, permuted as stage_x.  All of
// a thread's x (and norm) loads are issued before any is used: one memory round trip, not one
// per float4 (the wave's prefetched weight chunks were issued earlier, so the first use waits
// for those too).  J = float4 per thread (n <= 4 * J * PK_THREADS).
template <int E, int J>
__device__ __forceinline__ void pk_stage_j(const float* src, const int n, const void* norm_w, const int norm_dt,
                                           const float eps, float4* xs4, float* red) {
    const int tid = pk_tid();
    const int n4 = n >> 2;
    u32x4 u[J];
#pragma unroll
    for (int j = 0; j < J; j++) u[j] = ld_sc1_x4(src, (uint32_t)min(tid + j * PK_THREADS, n4 - 1) * 16);
    float4 w[J];
    if (norm_w) {
#pragma unroll
        for (int j = 0; j < J; j++) w[j] = load_norm4_nb(norm_w, norm_dt, n, min(tid + j * PK_THREADS, n4 - 1));
    }
    float scale = 1.f;
    if (norm_w) {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < J; j++) {
            const float d = bits_f32(u[j].x) * bits_f32(u[j].x) + bits_f32(u[j].y) * bits_f32(u[j].y) +
                            bits_f32(u[j].z) * bits_f32(u[j].z) + bits_f32(u[j].w) * bits_f32(u[j].w);
            ss += (tid + j * PK_THREADS < n4) ? d : 0.f;
        }
        ss = wave_sum(ss);
        if ((tid & 63) == 0) red[tid >> 6] = ss;
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int wv = 0; wv < PK_WAVES; wv++) tot += red[wv];
        scale = 1.0f / sqrtf(tot / (float)n + eps);
    }
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int i = min(tid + j * PK_THREADS, n4 - 1);  // duplicates store the same value
        float4 v = make_float4(bits_f32(u[j].x), bits_f32(u[j].y), bits_f32(u[j].z), bits_f32(u[j].w));
        if (norm_w) {
            v.x = v.x * scale * w[j].x;
            v.y = v.y * scale * w[j].y;
            v.z = v.z * scale * w[j].z;
            v.w = v.w * scale * w[j].w;
        }
        const int c = i << 2;
        const int it = c / (64 * E);
        const int rem = c - it * 64 * E;
        const int l = rem / E;
        const int qd = (rem - l * E) >> 2;
        xs4[(it * (E / 4) + qd) * 64 + l] = v;
    }
    __syncthreads();
}
template <int E>
__device__ __forceinline__ void pk_stage(const float* src, const int n, const void* norm_w, const int norm_dt,
                                         const float eps, float4* xs4, float* red) {
    if ((n >> 2) <= 2 * PK_THREADS) pk_stage_j<E, 2>(src, n, norm_w, norm_dt, eps, xs4, red);
    else if ((n >> 2) <= 4 * PK_THREADS) pk_stage_j<E, 4>(src, n, norm_w, norm_dt, eps, xs4, red);
    else pk_stage_j<E, 8>(src, n, norm_w, norm_dt, eps, xs4, red);  // host: n <= 4 * 8 * PK_THREADS
}

// Per-wave streaming state: the register chunk in flight and which group it belongs to.
struct PkStream {
    u32x4 buf[PK_U][PK_ROWS];
    int pre_group;       // group index whose chunk 0 is in buf, or -1
    const char* pre_w;   // matrix of that group
};

// Rows [r0, r1) of a matrix owned by this workgroup; wave w takes groups w, w + 16, ...
struct PkRange {
    const char* w;
    size_t rb;     // row bytes
    int n;         // row length (elements)
    int r0, r1;    // row range (r0 even)
};

// Request chunk 0 of this wave's first group of R.  buf is written on every path (zeros when
// the wave has no group), so the compiler sees it dead once pk_gemv has consumed it.
template <int DT>
__device__ __forceinline__ void pk_prefetch(PkStream& st, const PkRange& R) {
    constexpr int E = WDec<DT>::E;
    const int wid = pk_tid() >> 6, lane = pk_tid() & 63;
    const int g = R.r0 / PK_ROWS + wid;
    st.pre_group = -1;
    st.pre_w = R.w;
    if (g * PK_ROWS < R.r1 && R.n / (64 * E) >= PK_U) {
        const char* wrow = R.w + (size_t)g * PK_ROWS * R.rb + lane * 16;
        const size_t rs = (g * PK_ROWS + PK_ROWS - 1 < R.r1) ? R.rb : 0;
        gemv_load<PK_ROWS, PK_U, true>(st.buf, wrow, rs, 0);
        st.pre_group = g;
    } else {
#pragma unroll
        for (int u = 0; u < PK_U; u++)
#pragma unroll
            for (int r = 0; r < PK_ROWS; r++) st.buf[u][r] = u32x4{0u, 0u, 0u, 0u};
    }
}

// Chunks [it, n) of one group of rows, accumulated into acc.
template <int DT>
__device__ __forceinline__ void pk_rows(const char* wrow, const size_t rs, const int n, const float4* xs4, int it,
                                        const int lane, float* acc) {
    constexpr int E = WDec<DT>::E;
    const int n_full = n / (64 * E);
    const int n_it = (n + 64 * E - 1) / (64 * E);
    for (; it + PK_U <= n_full; it += PK_U) gemv_chunk<DT, PK_ROWS, PK_U, true>(wrow, rs, xs4, it, lane, acc);
    for (; it + 2 <= n_full; it += 2) gemv_chunk<DT, PK_ROWS, 2, true>(wrow, rs, xs4, it, lane, acc);
    for (; it < n_full; it++) gemv_chunk<DT, PK_ROWS, 1, true>(wrow, rs, xs4, it, lane, acc);
    if (it < n_it && (it * 64 + lane) * E < n) gemv_chunk<DT, PK_ROWS, 1, true>(wrow, rs, xs4, it, lane, acc);
}

// One gemv phase of this workgroup; `epi(row0, acc)` runs on lane 0 of each group.  The
// wave's first group starts from the prefetched chunk (peeled, so buf dies there).
template <int DT, class Epi>
__device__ __forceinline__ void pk_gemv(PkStream& st, const PkRange& R, const float4* xs4, Epi&& epi) {
    const int wid = pk_tid() >> 6, lane = pk_tid() & 63;
    int g = R.r0 / PK_ROWS + wid;
    if (g * PK_ROWS >= R.r1) return;
    {
        const int row0 = g * PK_ROWS;
        const size_t rs = (row0 + PK_ROWS - 1 < R.r1) ? R.rb : 0;
        const char* wrow = R.w + (size_t)row0 * R.rb + lane * 16;
        float acc[PK_ROWS];
#pragma unroll
        for (int r = 0; r < PK_ROWS; r++) acc[r] = 0.f;
        int it = 0;
        if (st.pre_group == g && st.pre_w == R.w) {
            gemv_compute<DT, PK_ROWS, PK_U>(st.buf, xs4, 0, lane, acc);
            it = PK_U;
        }
        st.pre_group = -1;
        pk_rows<DT>(wrow, rs, R.n, xs4, it, lane, acc);
#pragma unroll
        for (int r = 0; r < PK_ROWS; r++) acc[r] = wave_sum(acc[r]);
        if (lane == 0) epi(row0, acc);
    }
    for (g += PK_WAVES; g * PK_ROWS < R.r1; g += PK_WAVES) {
        const int row0 = g * PK_ROWS;
        const size_t rs = (row0 + PK_ROWS - 1 < R.r1) ? R.rb : 0;
        const char* wrow = R.w + (size_t)row0 * R.rb + lane * 16;
        float acc[PK_ROWS];
#pragma unroll
        for (int r = 0; r < PK_ROWS; r++) acc[r] = 0.f;
        pk_rows<DT>(wrow, rs, R.n, xs4, 0, lane, acc);
#pragma unroll
        for (int r = 0; r < PK_ROWS; r++) acc[r] = wave_sum(acc[r]);
        if (lane == 0) epi(row0, acc);
    }
}

__device__ __forceinline__ PkRange pk_range(const void* w, size_t rb, int n, int rows, int nblk, int b) {
    int per = (rows + nblk - 1) / nblk;
    per = (per + PK_ROWS - 1) / PK_ROWS * PK_ROWS;
    PkRange R;
    R.w = (const char*)w;
    R.rb = rb;
    R.n = n;
    R.r0 = min(rows, b * per);
    R.r1 = min(rows, R.r0 + per);
    return R;
}

// Attention of KV head g over slots [s*T, min(kv_len, s*T+T)) inside the persistent kernel:
// attn_split_kernel's math, with q/K/V read by sc1 loads (written earlier in this launch).
// The workgroup that completes head g (single split, or last to arrive) publishes its 4
// outputs and adds 1 to att_cnt.
template <int HD, int QPK>
__device__ __forceinline__ void pk_attention(const PkArgs& a, const PkLayer& ly, const int g, const int s, const int T,
                                             const int n_active, const int kv_len, char* work, int* flag,
                                             unsigned* att_cnt) {
    constexpr int LPR = HD / 8;
    constexpr int RPP = PK_THREADS / LPR;
    constexpr int NO = QPK * HD;
    float* red = (float*)work;                     // [WAVES][NO]
    float* ml = red + PK_WAVES * NO;               // [QPK][2]
    float* sc = ml + ((2 * QPK + 3) & ~3);         // [QPK][T]
    const int tid = pk_tid(), lane = tid & 63, wid = tid >> 6;
    const int sub = tid % LPR, rr = tid / LPR;
    const int t0 = s * T, t1 = min(kv_len, t0 + T);
    const float scale = 1.0f / sqrtf((float)HD);
    const uint32_t colb = (uint32_t)((g * HD + sub * 8) * 2);
    const uint32_t rowb = (uint32_t)a.kv_dim * 2;

    float qv[QPK][8];
#pragma unroll
    for (int h = 0; h < QPK; h++) {
        const float* qp = a.q + (size_t)(g * QPK + h) * HD + sub * 8;
        const u32x4 q0 = ld_sc1_x4(qp, 0), q1 = ld_sc1_x4(qp, 16);
        qv[h][0] = bits_f32(q0.x); qv[h][1] = bits_f32(q0.y); qv[h][2] = bits_f32(q0.z); qv[h][3] = bits_f32(q0.w);
        qv[h][4] = bits_f32(q1.x); qv[h][5] = bits_f32(q1.y); qv[h][6] = bits_f32(q1.z); qv[h][7] = bits_f32(q1.w);
    }
    // scores
    for (int base = t0; base < t1; base += ATTN_PREF * RPP) {
        u32x4 kk[ATTN_PREF];
#pragma unroll
        for (int p = 0; p < ATTN_PREF; p++) {
            const int t = base + rr + p * RPP;
            if (t < t1) kk[p] = ld_sc1_x4(ly.kc, (uint32_t)t * rowb + colb);
        }
#pragma unroll
        for (int p = 0; p < ATTN_PREF; p++) {
            const int t = base + rr + p * RPP;
            if (t < t1) {
                float kf[8];
                WDec<XH_F16>::dec(kk[p], kf);
#pragma unroll
                for (int h = 0; h < QPK; h++) {
                    float pr = 0.f;
#pragma unroll
                    for (int i = 0; i < 8; i++) pr = fmaf(qv[h][i], kf[i], pr);
                    pr = group_reduce<LPR>(pr);
                    if (sub == 0) sc[h * T + (t - t0)] = pr * scale;
                }
            }
        }
    }
    __syncthreads();
    const int len = t1 - t0;
    for (int h = wid; h < QPK; h += PK_WAVES) {
        float m = -FLT_MAX;
        for (int i = lane; i < len; i += 64) m = fmaxf(m, sc[h * T + i]);
        m = wave_max(m);
        float l = 0.f;
        for (int i = lane; i < len; i += 64) {
            const float e = expf(sc[h * T + i] - m);
            sc[h * T + i] = e;
            l += e;
        }
        l = wave_sum(l);
        if (lane == 0) { ml[2 * h] = m; ml[2 * h + 1] = l; }
    }
    __syncthreads();
    float acc[QPK][8];
#pragma unroll
    for (int h = 0; h < QPK; h++)
#pragma unroll
        for (int i = 0; i < 8; i++) acc[h][i] = 0.f;
    for (int base = t0; base < t1; base += ATTN_PREF * RPP) {
        u32x4 vv[ATTN_PREF];
#pragma unroll
        for (int p = 0; p < ATTN_PREF; p++) {
            const int t = base + rr + p * RPP;
            if (t < t1) vv[p] = ld_sc1_x4(ly.vc, (uint32_t)t * rowb + colb);
        }
#pragma unroll
        for (int p = 0; p < ATTN_PREF; p++) {
            const int t = base + rr + p * RPP;
            if (t < t1) {
                float vf[8];
                WDec<XH_F16>::dec(vv[p], vf);
#pragma unroll
                for (int h = 0; h < QPK; h++) {
                    const float e = sc[h * T + (t - t0)];
#pragma unroll
                    for (int i = 0; i < 8; i++) acc[h][i] = fmaf(e, vf[i], acc[h][i]);
                }
            }
        }
    }
#pragma unroll
    for (int h = 0; h < QPK; h++)
#pragma unroll
        for (int i = 0; i < 8; i++)
            acc[h][i] = strided_reduce<LPR>(acc[h][i]);
    if (lane < LPR) {
#pragma unroll
        for (int h = 0; h < QPK; h++)
#pragma unroll
            for (int i = 0; i < 8; i++) red[wid * NO + h * HD + sub * 8 + i] = acc[h][i];
    }
    __syncthreads();
    auto block_sum = [&](const int idx) {
        float o = 0.f;
#pragma unroll
        for (int w = 0; w < PK_WAVES; w++) o += red[w * NO + idx];
        return o;
    };
    if (n_active == 1) {
        for (int idx = tid; idx < NO; idx += PK_THREADS)
            st_sc1_f(a.attn + (size_t)g * NO + idx, block_sum(idx) / ml[2 * (idx / HD) + 1]);
        pk_signal(att_cnt);
        return;
    }
    float* po = a.part_o + ((size_t)s * a.n_heads + g * QPK) * HD;
    for (int idx = tid; idx < NO; idx += PK_THREADS) st_sc1_f(po + idx, block_sum(idx));
    if (tid < 2 * QPK) st_sc1_f(a.part_ml + ((size_t)s * a.n_heads + g * QPK) * 2 + tid, ml[tid]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int ticket = __hip_atomic_fetch_add(a.tickets + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = ticket == n_active - 1;
        if (last) __hip_atomic_store(a.tickets + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
    }
    __syncthreads();
    const int last = *flag;
    __syncthreads();
    if (!last) return;
    float* wts = sc;
    for (int h = wid; h < QPK; h += PK_WAVES) {
        float mv[2] = {-FLT_MAX, -FLT_MAX}, lv[2] = {0.f, 0.f};
        int c = 0;
        for (int j = lane; j < n_active; j += 64, c++) {
            const float* mlp = a.part_ml + ((size_t)j * a.n_heads + g * QPK + h) * 2;
            mv[c & 1] = ld_sc1_f(mlp);
            lv[c & 1] = ld_sc1_f(mlp + 1);
        }
        const float M = wave_max(fmaxf(mv[0], mv[1]));
        float den = 0.f;
        c = 0;
        for (int j = lane; j < n_active; j += 64, c++) {
            const float f = expf(mv[c & 1] - M);
            wts[h * n_active + j] = f;
            den = fmaf(f, lv[c & 1], den);
        }
        den = wave_sum(den);
        if (lane == 0) red[h] = den;
    }
    __syncthreads();
    for (int idx = tid; idx < NO; idx += PK_THREADS) {
        const int h = idx / HD;
        const float* w = wts + h * n_active;
        const float* src = a.part_o + (size_t)g * NO + idx;
        const size_t stride = (size_t)a.n_heads * HD;
        float num = 0.f;
        int j = 0;
        for (; j + 4 <= n_active; j += 4) {
            const float p0 = ld_sc1_f(src + (j + 0) * stride), p1 = ld_sc1_f(src + (j + 1) * stride);
            const float p2 = ld_sc1_f(src + (j + 2) * stride), p3 = ld_sc1_f(src + (j + 3) * stride);
            num = fmaf(w[j], p0, num);
            num = fmaf(w[j + 1], p1, num);
            num = fmaf(w[j + 2], p2, num);
            num = fmaf(w[j + 3], p3, num);
        }
        for (; j < n_active; j++) num = fmaf(w[j], ld_sc1_f(src + j * stride), num);
        st_sc1_f(a.attn + (size_t)g * NO + idx, num / red[h]);
    }
    pk_signal(att_cnt);
}


template <int DT, int DTC, int HD, int QPK>
__global__ __launch_bounds__(PK_THREADS) void persistent_decode_kernel(const PkArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* red = (float*)smem;                 // 16 floats
    int* flag = (int*)(smem + 128);            // LDS broadcast words
    unsigned long long* kred = (unsigned long long*)(smem + 256);  // [PK_WAVES]
    char* work = smem + 512;                   // x image / attention tiles
    float4* xs4 = (float4*)work;
    constexpr int E = WDec<DT>::E;
    constexpr int EC = WDec<DTC>::E;

    const int nblk = gridDim.x, b = blockIdx.x;
    const int tid = pk_tid(), lane = tid & 63, wid = tid >> 6;
    const int L = a.n_layers;
    const int esz = (int)(16 / E);  // bytes per element of the matrices
    const int escz = (int)(16 / EC);

    PkStream st;
    st.pre_group = -1;
    st.pre_w = nullptr;

    // x rows owned by this workgroup (same partition as Wo / W2 rows)
    const PkRange xr = pk_range(nullptr, 0, 0, a.dim, nblk, b);

    const int n_tok = a.n_prompt + a.n_gen;
    unsigned cls_done = 0;
    int token = -1;
    bool alive = true;

    // decode from existing logits (left by the previous launch): first token = their argmax
    if (a.n_prompt == 0 && n_tok > 0) {
        unsigned long long best = 0;
        for (int i = tid; i < a.vocab; i += PK_THREADS) {
            const float v = a.logits[i];
            if (v > FLT_MIN) {
                const unsigned long long k = pk_key(v, i);
                best = k > best ? k : best;
            }
        }
        // block reduce
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long other = __shfl_xor(best, o, 64);
            best = other > best ? other : best;
        }
        if (lane == 0) kred[wid] = best;
        __syncthreads();
        best = 0;
        for (int w = 0; w < PK_WAVES; w++) best = kred[w] > best ? kred[w] : best;
        __syncthreads();
        token = best ? (int)(~(uint32_t)best) : 0;
    }

    for (int t = 0; t < n_tok && alive; t++) {
        const int tid = pk_tid();
        const PkArgs& a = *pk_args();
        const int pos = a.pos0 + t;
        if (t < a.n_prompt) token = a.prompt[t];
        const bool gen = t >= a.n_prompt;  // token produced by argmax
        if (gen && b == 0 && tid == 0) {
            a.tokens_out[t - a.n_prompt] = token;
            *a.n_done = t - a.n_prompt + 1;
        }
        if (gen && (token == a.stop_a || token == a.stop_b)) break;
        const int msl = a.max_seq_len;
        const int kv_sink = pos >= msl ? 2 : 0;
        const int kv_pos = kv_sink + (pos - kv_sink) % (msl - kv_sink);
        const int kv_len = pos >= msl ? msl : pos + 1;
        const bool want_logits = (t == n_tok - 1) ? a.logits_last != 0 : (t >= a.n_prompt - 1);
        const int trw = !a.trace || t != n_tok - 1 ? -1 : b == 0 ? 0 : b == nblk / 2 ? 1 : b == nblk - 1 ? 2 : -1;
#define PK_TR(l_, ph_, k_)                                                                                 \
    do {                                                                                                   \
        if (trw >= 0 && pk_tid() == 0)                                                                     \
            pk_args()->trace[trw * pk_trace_len(L) + ((l_) * PK_PHASES + (ph_)) * 2 + (k_)] = pk_now();    \
    } while (0)
        PK_TR(L, 1, 1);

        // ---- embedding: own rows of x, and layer 0's input image straight from the row ----
        for (int r = xr.r0 + tid; r < xr.r1; r += PK_THREADS)
            st_sc1_f(a.x + r, dec1(a.embed_dt, a.embed, (size_t)token * a.dim + r));

        for (int l = 0; l < L && alive; l++) {
            const int tid = pk_tid(), lane = tid & 63, wid = tid >> 6;
            const PkArgs& a = *pk_args();
            const PkLayer& ly = a.layers[l];
            unsigned* cnt = a.counters + l * PK_PHASES;
            const unsigned tgt = (unsigned)(t + 1) * nblk;

            // ===== QKV =====
            const PkRange rq = pk_range(ly.wqkv, (size_t)a.dim * esz, a.dim, a.q_dim + 2 * a.kv_dim, nblk, b);
            if (st.pre_w != rq.w) pk_prefetch<DT>(st, rq);
            if (l == 0) {
                // input = rmsnorm(embed row): stage from the embedding table directly
                float ss = 0.f;
                for (int i = tid; i < (a.dim >> 2); i += PK_THREADS) {
                    float4 v;
                    const size_t base = (size_t)token * a.dim + 4 * i;
                    v.x = dec1(a.embed_dt, a.embed, base);
                    v.y = dec1(a.embed_dt, a.embed, base + 1);
                    v.z = dec1(a.embed_dt, a.embed, base + 2);
                    v.w = dec1(a.embed_dt, a.embed, base + 3);
                    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                    const int c = i << 2, it = c / (64 * E), rem = c - it * 64 * E, lq = rem / E,
                              qd = (rem - lq * E) >> 2;
                    xs4[(it * (E / 4) + qd) * 64 + lq] = v;
                }
                ss = wave_sum(ss);
                if (lane == 0) red[wid] = ss;
                __syncthreads();
                float tot = 0.f;
                for (int w = 0; w < PK_WAVES; w++) tot += red[w];
                const float scale = 1.0f / sqrtf(tot / (float)a.dim + a.eps);
                for (int i = tid; i < (a.dim >> 2); i += PK_THREADS) {
                    const int c = i << 2, it = c / (64 * E), rem = c - it * 64 * E, lq = rem / E,
                              qd = (rem - lq * E) >> 2;
                    float4& v = xs4[(it * (E / 4) + qd) * 64 + lq];
                    const float4 wn = load_norm4(ly.attn_norm, a.norm_dt, i);
                    v.x = v.x * scale * wn.x;
                    v.y = v.y * scale * wn.y;
                    v.z = v.z * scale * wn.z;
                    v.w = v.w * scale * wn.w;
                }
                __syncthreads();
            } else {
                if (!(alive = pk_wait(a.counters + (l - 1) * PK_PHASES + 4, tgt, a.err, flag))) break;
                PK_TR(l, 0, 0);
                pk_stage<E>(a.x, a.dim, ly.attn_norm, a.norm_dt, a.eps, xs4, red);
            }
            // sink re-rotation (src/infer.cpp:421-431), workgroup 0
            if (b == 0 && kv_sink) {
                for (int r = 0; r < kv_sink; r++) {
                    uint16_t* krow = ly.kc + (size_t)r * a.kv_dim;
                    for (int p = tid; p < (a.kv_dim >> 1); p += PK_THREADS) {
                        const int i = p << 1;
                        const int jh = (i % a.head_dim) >> 1;
                        const uint32_t pr = ld_sc1_u32(krow + i);
                        const float k0 = f16_bits_to_f32((uint16_t)(pr & 0xffffu));
                        const float k1 = f16_bits_to_f32((uint16_t)(pr >> 16));
                        const float fcr = a.sink_cos[jh], fci = a.sink_sin[jh];
                        const uint32_t o = (uint32_t)f32_to_f16_bits(k0 * fcr - k1 * fci) |
                                           ((uint32_t)f32_to_f16_bits(k0 * fci + k1 * fcr) << 16);
                        st_sc1_u32(krow + i, o);
                    }
                }
            }
            pk_gemv<DT>(st, rq, xs4, [&](const int row0, const float* acc) {
#pragma unroll
                for (int p = 0; p < PK_ROWS; p += 2) {
                    const int row = row0 + p;
                    float v0 = clipf(acc[p], a.qkv_clip), v1 = clipf(acc[p + 1], a.qkv_clip);
                    if (row < a.q_dim) {
                        rope_pair(v0, v1, row, a.head_dim, pos, a.rope_freq);
                        st_sc1_f(a.q + row, v0);
                        st_sc1_f(a.q + row + 1, v1);
                    } else {
                        const bool isk = row < a.q_dim + a.kv_dim;
                        const int r = isk ? row - a.q_dim : row - a.q_dim - a.kv_dim;
                        if (isk) rope_pair(v0, v1, r, a.head_dim, pos, a.rope_freq);
                        uint16_t* dst = (isk ? ly.kc : ly.vc) + (size_t)kv_pos * a.kv_dim + r;
                        st_sc1_u32(dst, (uint32_t)f32_to_f16_bits(v0) | ((uint32_t)f32_to_f16_bits(v1) << 16));
                    }
                }
            });
            pk_signal(cnt + 0);
            PK_TR(l, 0, 1);

            // ===== attention =====
            // workgroups without attention work request their Wo rows right away; the others
            // after their attention (holding them across it would spill)
            const PkRange ro = pk_range(ly.wo, (size_t)a.q_dim * esz, a.q_dim, a.dim, nblk, b);
            {
                const int T = attn_split_len(kv_len, a.nsplit);
                const int nact = (kv_len + T - 1) / T;
                const int nwork = a.n_kv_heads * nact;
                if (b < nwork) {
                    if (!(alive = pk_wait(cnt + 0, tgt, a.err, flag))) break;
                    const int g = b / nact, s = b - g * nact;
                    PK_TR(l, 1, 0);
                    pk_attention<HD, QPK>(a, ly, g, s, T, nact, kv_len, work, flag, cnt + 1);
                    PK_TR(l, 1, 1);
                }
            }
            pk_prefetch<DT>(st, ro);

            // ===== Wo (+ residual) =====
            if (!(alive = pk_wait(cnt + 1, (unsigned)(t + 1) * a.n_kv_heads, a.err, flag))) break;
            PK_TR(l, 2, 0);
            pk_stage<E>(a.attn, a.q_dim, nullptr, 0, 0.f, xs4, red);
            pk_gemv<DT>(st, ro, xs4, [&](const int row0, const float* acc) {
#pragma unroll
                for (int r = 0; r < PK_ROWS; r++)
                    if (row0 + r < ro.r1) st_sc1_f(a.x + row0 + r, ld_sc1_f(a.x + row0 + r) + acc[r]);
            });
            const PkRange r13 = pk_range(ly.w13, (size_t)a.dim * esz, a.dim, 2 * a.hidden, nblk, b);
            pk_prefetch<DT>(st, r13);
            pk_signal(cnt + 2);
            PK_TR(l, 2, 1);

            // ===== W1/W3 (+ rmsnorm, act * up) =====
            if (!(alive = pk_wait(cnt + 2, tgt, a.err, flag))) break;
            PK_TR(l, 3, 0);
            pk_stage<E>(a.x, a.dim, ly.ffn_norm, a.norm_dt, a.eps, xs4, red);
            pk_gemv<DT>(st, r13, xs4, [&](const int row0, const float* acc) {
#pragma unroll
                for (int p = 0; p < PK_ROWS; p += 2) st_sc1_f(a.hb + ((row0 + p) >> 1), act_fn(a.act, acc[p]) * acc[p + 1]);
            });
            const PkRange r2 = pk_range(ly.w2, (size_t)a.hidden * esz, a.hidden, a.dim, nblk, b);
            pk_prefetch<DT>(st, r2);
            pk_signal(cnt + 3);
            PK_TR(l, 3, 1);

            // ===== W2 (+ residual) =====
            if (!(alive = pk_wait(cnt + 3, tgt, a.err, flag))) break;
            PK_TR(l, 4, 0);
            pk_stage<E>(a.hb, a.hidden, nullptr, 0, 0.f, xs4, red);
            pk_gemv<DT>(st, r2, xs4, [&](const int row0, const float* acc) {
#pragma unroll
                for (int r = 0; r < PK_ROWS; r++)
                    if (row0 + r < r2.r1) st_sc1_f(a.x + row0 + r, ld_sc1_f(a.x + row0 + r) + acc[r]);
            });
            if (l + 1 < L) {
                const PkLayer& nx = a.layers[l + 1];
                pk_prefetch<DT>(st, pk_range(nx.wqkv, (size_t)a.dim * esz, a.dim, a.q_dim + 2 * a.kv_dim, nblk, b));
            }
            pk_signal(cnt + 4);
            PK_TR(l, 4, 1);
        }
        if (!alive) break;

        // ===== final rmsnorm + lm_head (+ argmax candidates) =====
        if (want_logits) {
            const int tid = pk_tid(), lane = tid & 63, wid = tid >> 6;
            const PkArgs& a = *pk_args();
            const PkRange rc = pk_range(a.wcls, (size_t)a.dim * escz, a.dim, a.vocab, nblk, b);
            pk_prefetch<DTC>(st, rc);
            if (!(alive = pk_wait(a.counters + (L - 1) * PK_PHASES + 4, (unsigned)(t + 1) * nblk, a.err, flag))) break;
            PK_TR(L, 0, 0);
            pk_stage<EC>(a.x, a.dim, a.final_norm, a.norm_dt, a.eps, xs4, red);
            // Sampler::sample_argmax semantics: only logits > FLT_MIN compete (src/sampler.cpp:19-30)
            unsigned long long best = 0;
            pk_gemv<DTC>(st, rc, xs4, [&](const int row0, const float* acc) {
#pragma unroll
                for (int r = 0; r < PK_ROWS; r++)
                    if (row0 + r < rc.r1) {
                        a.logits[row0 + r] = acc[r];
                        if (acc[r] > FLT_MIN) {
                            const unsigned long long k = pk_key(acc[r], row0 + r);
                            best = k > best ? k : best;
                        }
                    }
            });
            // the next token's first weights do not depend on the argmax
            if (t + 1 < n_tok)
                pk_prefetch<DT>(st, pk_range(a.layers[0].wqkv, (size_t)a.dim * esz, a.dim, a.q_dim + 2 * a.kv_dim,
                                             nblk, b));
            // lane 0 of each wave holds its best; reduce over waves
            if (lane == 0) kred[wid] = best;
            __syncthreads();
            if (tid == 0) {
                unsigned long long bb = 0;
                for (int w = 0; w < PK_WAVES; w++) bb = kred[w] > bb ? kred[w] : bb;
                __hip_atomic_store(a.cand + b, bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            cls_done++;
            pk_signal(a.counters + L * PK_PHASES);
            PK_TR(L, 0, 1);
            if (t + 1 < n_tok && t + 1 >= a.n_prompt) {
                // next token = argmax over all workgroups' candidates (same in every workgroup)
                if (!(alive = pk_wait(a.counters + L * PK_PHASES, cls_done * nblk, a.err, flag))) break;
                unsigned long long bb = 0;
                for (int i = tid; i < nblk; i += PK_THREADS) {
                    const unsigned long long k =
                        __hip_atomic_load(a.cand + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bb = k > bb ? k : bb;
                }
                for (int o = 32; o > 0; o >>= 1) {
                    const unsigned long long other = __shfl_xor(bb, o, 64);
                    bb = other > bb ? other : bb;
                }
                __syncthreads();
                if (lane == 0) kred[wid] = bb;
                __syncthreads();
                bb = 0;
                for (int w = 0; w < PK_WAVES; w++) bb = kred[w] > bb ? kred[w] : bb;
                __syncthreads();
                token = bb ? (int)(~(uint32_t)bb) : 0;
                PK_TR(L, 1, 0);
            }
        }
    }
}

#undef PK_TR

}  // namespace xalm
