// attn_wo.h — attention and the Wo projection (+ residual) in ONE launch.
//
// Same math as attn_split_kernel followed by gemv_kernel<PRO_PLAIN, EPI_RESID> (the head loop
// and output projection of Block::_block_cpu, jubruckne/Xalm src/infer.cpp:434-452), with the
// launch boundary between them replaced by an in-launch hand-off:
// * workgroups [0, n_kv_heads * nsplit) are attention workgroups (KV head g = b / nsplit,
//   split s = b % nsplit; splits past kv_len exit at once).  Every active split stores its
//   partial (o, m, l) write-through (sc1), drains, and adds 1 to sync[0]: the attention chain
//   is one K/V round trip plus one publish, with no split waiting on another;
// * the remaining workgroups own the Wo rows.  Each wave requests its first U weight chunks
//   (the whole row for f16 / bf16 at d = 4096: the Wo matrix is in flight across the chip)
//   BEFORE waiting, so the 33.5 MB weight stream overlaps the attention instead of following
//   it; one lane polls sync[0] until all n_kv_heads * n_active splits are published (relaxed
//   loads, s_sleep, 2 s bound), then the workgroup merges the partials while staging its x
//   image (out = sum_s e^{m_s-M} o_s / sum_s e^{m_s-M} l_s, as attention.h's merge) with sc1
//   loads, and finishes the rows;
// * the next launch on the stream (W1/W3 of the layer, GemvArgs::aw_reset) zeroes sync[] for
//   the next use.
// Attention workgroups are dispatched first (lowest block ids) and never wait on anything, so
// progress does not depend on co-residency.  Fan-in: n_kv_heads * n_active arrivals.
#pragma once

#include "attention.h"
#include "gemv.h"

namespace xalm {

#ifndef AW_THREADS_OVERRIDE
constexpr int AW_THREADS = 1024;  // 16 waves: one workgroup per CU at <= 128 VGPRs
#else
constexpr int AW_THREADS = AW_THREADS_OVERRIDE;
#endif
// Wo shape: 2 rows per wave, a 4096-long f16 / bf16 row (8 KiB) or fp8 row (4 KiB) in U chunks
template <int DT>
using AwShape = GemvShape<AW_THREADS, 2, (WDec<DT>::E >= 16 ? 4 : 8), true, 4, true>;

// sync (AW_SYNC_WORDS per layer): [0] head arrivals, [2] timeout flag (sticky, host-checked),
// [AW_FLAG0 + 32 k] "heads done" flag of XCD k: set by the last head arrival, polled by that
// XCD's Wo workgroups (one polled line per XCD instead of every Wo workgroup polling the
// counter the arrivals add to).  Words 0, 32, ..., 32 (AW_RESET_WORDS - 1) are zeroed by the
// next launch.
constexpr int AW_FLAG0 = 32;
constexpr int AW_SYNC_WORDS = AW_FLAG0 + 8 * 32;
static_assert(AW_SYNC_WORDS == 32 * AW_RESET_WORDS, "every hand-off word is reset");

// More than MAXS partials per head to merge (aw_stage_merged keeps MAXS in registers beside
// the Wo rows): the attention side merges instead (attn_block SIGNAL), so a Wo workgroup
// reads one merged vector, not n_active partials per element.
constexpr int AW_MAXS = 4;
#ifndef AW_EARLY_WAVE0
#define AW_EARLY_WAVE0 1
#endif
template <int HD>
__device__ __forceinline__ bool aw_long(const AttnArgs& aa) {
    const int kv_len = aa.sp->kv_len;
    const int T = attn_split_len(kv_len, aa.nsplit, attn_min_t_partials(HD, AW_THREADS));
    return (kv_len + T - 1) / T > AW_MAXS;
}
template <int E>
__host__ __device__ constexpr size_t aw_image_bytes(const int n) {
    return (size_t)((n + 64 * E - 1) / (64 * E)) * 64 * E * sizeof(float);
}

#ifndef AW_STAGE_NA
#define AW_STAGE_NA 1
#endif
// aw_stage_merged's register path for NA partials: per thread its float4 of each partial and its
// head's (m, l) pairs (one 8-byte load each), merged in partial order
template <int E, int HD, int NA, int THREADS>
__device__ __forceinline__ void aw_stage_na(const AttnArgs& aa, const int n, float4* xs4) {
    const int nh = aa.n_heads;
    const size_t stride = (size_t)nh * HD;  // floats per split in part_o
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)aa.part_ml, 0, 0x7fffffff, 0x00020000);
    for (int i = threadIdx.x; i < (n >> 2); i += THREADS) {
        const int h = (4 * i) / HD;
        u32x4 ov[NA];
        uint32_t mlv[NA][2];
#pragma unroll
        for (int j = 0; j < NA; j++) {
            ov[j] = ld_sc1_x4(aa.part_o, (uint32_t)((j * stride + 4 * (size_t)i) * 4));
            const auto u = __builtin_amdgcn_raw_buffer_load_b64(rs, (j * nh + h) * 8, 0, 16);  // sc1
            mlv[j][0] = u[0];
            mlv[j][1] = u[1];
        }
        // out = sum_s e^{m_s-M} o_s / sum_s e^{m_s-M} l_s   (as attention.h's merge)
        float M = -FLT_MAX;
#pragma unroll
        for (int j = 0; j < NA; j++) M = fmaxf(M, bits_f32(mlv[j][0]));
        float den = 0.f;
        float4 num = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < NA; j++) {
            const float f = expf(bits_f32(mlv[j][0]) - M);
            den = fmaf(f, bits_f32(mlv[j][1]), den);
            num.x = fmaf(f, bits_f32(ov[j].x), num.x);
            num.y = fmaf(f, bits_f32(ov[j].y), num.y);
            num.z = fmaf(f, bits_f32(ov[j].z), num.z);
            num.w = fmaf(f, bits_f32(ov[j].w), num.w);
        }
        const float4 v = make_float4(num.x / den, num.y / den, num.z / den, num.w / den);
        const int c = i << 2;
        const int it = c / (64 * E);
        const int rem = c - it * 64 * E;
        const int l = rem / E;
        const int qd = (rem - l * E) >> 2;
        xs4[(it * (E / 4) + qd) * 64 + l] = v;
    }
}

// x image of the Wo rows = the merged attention output.  Up to AW_MAXS partials (attn_wo.h: longer
// histories arrive merged, aw_long) every thread loads its float4 of each partial AND its head's
// (m, l) pairs in one round trip and forms the weights itself (n_active expf per thread): no LDS
// exchange and no barrier between the loads and the image.  More partials: wts (LDS
// [n_heads][n_active] weights, [n_heads] denominators, then the (m, l) pairs) shared per head.
template <int E, int HD, int THREADS = AW_THREADS>
__device__ __forceinline__ void aw_stage_merged(const AttnArgs& aa, const int n, const int n_active, float4* xs4,
                                                float* wts) {
    constexpr int MAXS = AW_MAXS;
    const int tid = threadIdx.x;
    const int nh = aa.n_heads;
    const int n4 = n >> 2;
    const size_t stride = (size_t)nh * HD;  // floats per split in part_o
    if (n_active > MAXS) {
        float* ml = wts + nh * (n_active + 1);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)aa.part_ml, 0, 0x7fffffff, 0x00020000);
        for (int i = tid; i < n_active * nh; i += THREADS) {
            ml[2 * i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, i * 8, 0, 16));  // sc1
            ml[2 * i + 1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, i * 8 + 4, 0, 16));
        }
        __syncthreads();
        // per head: weights e^{m_s - M} and the denominator sum_s e^{m_s - M} l_s
        for (int h = tid; h < nh; h += THREADS) {
            float M = -FLT_MAX;
            for (int j = 0; j < n_active; j++) M = fmaxf(M, ml[2 * (j * nh + h)]);
            float den = 0.f;
            for (int j = 0; j < n_active; j++) {
                const float f = expf(ml[2 * (j * nh + h)] - M);
                wts[h * n_active + j] = f;
                den = fmaf(f, ml[2 * (j * nh + h) + 1], den);
            }
            wts[nh * n_active + h] = den;
        }
        __syncthreads();
        for (int i = tid; i < n4; i += THREADS) {
            const int h = (4 * i) / HD;
            const float* w = wts + h * n_active;
            float4 num = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int j = 0; j < n_active; j++) {
                const u32x4 u = ld_sc1_x4(aa.part_o, (uint32_t)((j * stride + 4 * (size_t)i) * 4));
                num.x = fmaf(w[j], bits_f32(u.x), num.x);
                num.y = fmaf(w[j], bits_f32(u.y), num.y);
                num.z = fmaf(w[j], bits_f32(u.z), num.z);
                num.w = fmaf(w[j], bits_f32(u.w), num.w);
            }
            const float den = wts[nh * n_active + h];
            const float4 v = make_float4(num.x / den, num.y / den, num.z / den, num.w / den);
            const int c = i << 2;
            const int it = c / (64 * E);
            const int rem = c - it * 64 * E;
            const int l = rem / E;
            const int qd = (rem - l * E) >> 2;
            xs4[(it * (E / 4) + qd) * 64 + l] = v;
        }
        return;
    }
#if AW_STAGE_NA
    // the partial count as a constant: no clamped duplicate loads (n_active = 1 issued 4 o and
    // 8 (m, l) loads per thread for 1 and 2 it needs)
    switch (n_active) {
        case 1: aw_stage_na<E, HD, 1, THREADS>(aa, n, xs4); return;
        case 2: aw_stage_na<E, HD, 2, THREADS>(aa, n, xs4); return;
        case 3: aw_stage_na<E, HD, 3, THREADS>(aa, n, xs4); return;
        default: aw_stage_na<E, HD, MAXS, THREADS>(aa, n, xs4); return;
    }
#else
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)aa.part_ml, 0, 0x7fffffff, 0x00020000);
    for (int i = tid; i < n4; i += THREADS) {
        const int h = (4 * i) / HD;
        u32x4 ov[MAXS];
        float mv[MAXS], lv[MAXS];
#pragma unroll
        for (int j = 0; j < MAXS; j++) {  // clamped: every load in one basic block
            const int jj = j < n_active ? j : n_active - 1;
            ov[j] = ld_sc1_x4(aa.part_o, (uint32_t)((jj * stride + 4 * (size_t)i) * 4));
            const int mo = (jj * nh + h) * 8;
            mv[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, mo, 0, 16));  // sc1
            lv[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, mo + 4, 0, 16));
        }
        // out = sum_s e^{m_s-M} o_s / sum_s e^{m_s-M} l_s   (as attention.h's merge)
        float M = -FLT_MAX;
#pragma unroll
        for (int j = 0; j < MAXS; j++) M = j < n_active ? fmaxf(M, mv[j]) : M;
        float den = 0.f;
        float4 num = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < MAXS; j++) {
            if (j < n_active) {
                const float f = expf(mv[j] - M);
                den = fmaf(f, lv[j], den);
                num.x = fmaf(f, bits_f32(ov[j].x), num.x);
                num.y = fmaf(f, bits_f32(ov[j].y), num.y);
                num.z = fmaf(f, bits_f32(ov[j].z), num.z);
                num.w = fmaf(f, bits_f32(ov[j].w), num.w);
            }
        }
        const float4 v = make_float4(num.x / den, num.y / den, num.z / den, num.w / den);
        const int c = i << 2;
        const int it = c / (64 * E);
        const int rem = c - it * 64 * E;
        const int l = rem / E;
        const int qd = (rem - l * E) >> 2;
        xs4[(it * (E / 4) + qd) * 64 + l] = v;
    }
#endif
}

// x image of the Wo rows from the merged attention output (sc1: written in this launch)
template <int E>
__device__ __forceinline__ void aw_stage_out(const float* src, const int n, float4* xs4) {
    for (int i = threadIdx.x; i < (n >> 2); i += AW_THREADS) {
        const u32x4 u = ld_sc1_x4(src, (uint32_t)i * 16);
        const int c = i << 2;
        const int it = c / (64 * E);
        const int rem = c - it * 64 * E;
        const int l = rem / E;
        const int qd = (rem - l * E) >> 2;
        xs4[(it * (E / 4) + qd) * 64 + l] = make_float4(bits_f32(u.x), bits_f32(u.y), bits_f32(u.z), bits_f32(u.w));
    }
}

// trace (debug, null = off): per workgroup [8]: start, attention done | hand-off passed, end;
// attention workgroups also [2] split known, [3] scores done, [4] p.V done, [5] partial drained
template <int DT, int HD, int QPK>
__global__ __launch_bounds__(AW_THREADS) void attn_wo_kernel(const AttnArgs aa, const GemvArgs ga,
                                                                  const int n_kv_heads, unsigned* sync,
                                                                  unsigned long long* trace) {
    using S = AwShape<DT>;
    constexpr int E = WDec<DT>::E;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int n_att = n_kv_heads * aa.nsplit;
    const int b = blockIdx.x;
    if (trace && threadIdx.x == 0) trace[8 * b] = __builtin_amdgcn_s_memrealtime();
    const int kv_len = aa.sp->kv_len;
    const int T = attn_split_len(kv_len, aa.nsplit, attn_min_t_partials(HD, AW_THREADS));
    const int n_active = (kv_len + T - 1) / T;
    const bool merged = aw_long<HD>(aa);  // heads arrive merged (one arrival per KV head)
    const unsigned target = (unsigned)(merged ? n_kv_heads : n_kv_heads * n_active);
    if (b < n_att) {
        const int g = b / aa.nsplit, s = b - g * aa.nsplit;
        if (s >= n_active) return;  // a split past kv_len
        auto arrive = [&](unsigned* c) {
            const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1 == target) {
#pragma unroll
                for (int k = 0; k < 8; k++)
                    __hip_atomic_store(c + AW_FLAG0 + 32 * k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        };
        if (merged) {
            // long contexts: each KV head's last split merges (ticket) and signals the head
            attn_block<HD, QPK, AW_THREADS, false, attn_min_t_partials(HD, AW_THREADS), NoWait,
                       decltype(arrive), true>(aa, g, s, smem, sync, nullptr, NoWait(), arrive);
        } else {
            attn_block<HD, QPK, AW_THREADS, true, 0, NoWait, decltype(arrive)>(
                aa, g, s, smem, sync, trace ? trace + 8 * b : nullptr, NoWait(), arrive);
        }
        if (trace && threadIdx.x == 0) trace[8 * b + 1] = __builtin_amdgcn_s_memrealtime();
        return;
    }
    float4* xs4 = (float4*)(smem + LDS_HEAD_BYTES);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nb = gridDim.x - n_att;
    const int g = (b - n_att) * S::WAVES + wid;
    auto wait_heads = [&]() {
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            int xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 3)" : "=s"(xcc));
            const unsigned* flag = sync + AW_FLAG0 + 32 * (xcc & 7);
            while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz: flag, go on
                    __hip_atomic_store(sync + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        __syncthreads();
        if (trace && threadIdx.x == 0) trace[8 * b + 1] = __builtin_amdgcn_s_memrealtime();
        if (merged) aw_stage_out<E>(aa.out, ga.n, xs4);
        else aw_stage_merged<E, HD>(aa, ga.n, n_active, xs4, (float*)(smem + LDS_HEAD_BYTES + aw_image_bytes<E>(ga.n)));
        __syncthreads();
        if (trace && threadIdx.x == 0) trace[8 * b + 3] = __builtin_amdgcn_s_memrealtime();
    };
    const int n_groups = gemv_groups<S>(ga);
    if (ga.n == S::U * 64 * E && n_groups <= nb * S::WAVES) {
        // every wave owns at most one group and its whole rows fit the U chunks: request them,
        // then wait; nothing but the dot products is left after the hand-off
        // wave 0 polls, so it requests its rows only after the hand-off: a poll's sc1 load
        // completes in order behind the polling wave's own outstanding loads (vmcnt)
        u32x4 w[S::U][S::ROWS];
        float xres[S::ROWS];
        auto fetch = [&]() {
            gemv_prefetch<S>(ga, g, lane, w);
            if (lane == 0) {
#pragma unroll
                for (int r = 0; r < S::ROWS; r++) xres[r] = g * S::ROWS + r < ga.rows ? ga.out[g * S::ROWS + r] : 0.f;
            }
        };
        // every wave requests its Wo rows before the hand-off, wave 0 too: its poll's sc1 loads
        // complete behind its own row loads (vmcnt is in order), but those land (≈5 µs at
        // full HBM rate) before the heads are done, while rows requested after the hand-off
        // made wave 0 the launch's last wave by ≈1.5 µs
        const bool early = AW_EARLY_WAVE0 || wid != 0;
        if (g < n_groups && early) fetch();
        wait_heads();
        if (g < n_groups && !early) fetch();
        if (g < n_groups) {
            float acc[S::ROWS];
#pragma unroll
            for (int r = 0; r < S::ROWS; r++) acc[r] = 0.f;
            gemv_compute<DT, S::ROWS, S::U>(w, xs4, 0, lane, acc);
#pragma unroll
            for (int r = 0; r < S::ROWS; r++) acc[r] = wave_sum(acc[r]);
            if (lane == 0) {
#pragma unroll
                for (int r = 0; r < S::ROWS; r++)  // x += Wo . attn (src/infer.cpp:449-452)
                    if (g * S::ROWS + r < ga.rows) ga.out[g * S::ROWS + r] = xres[r] + acc[r];
            }
        }
    } else {
        using G = GemvShape<AW_THREADS, S::ROWS, 4, true, 4, false>;
        wait_heads();
        u32x4 none[G::U][G::ROWS];
        gemv_rows<DT, EPI_RESID, G, false>(ga, g, nb * S::WAVES, lane, xs4, none);
    }
    if (trace) {
        __syncthreads();
        if (threadIdx.x == 0) trace[8 * b + 2] = __builtin_amdgcn_s_memrealtime();
    }
    // sync[0] and the flags are zeroed by the next launch on the stream (the W1/W3 matvec of
    // this layer, GemvArgs::aw_reset): no returning ticket atomic at the end of every Wo
    // workgroup (a round trip on the launch's tail)
}

// LDS bytes: the larger of the attention tiles (at AW_THREADS) and the Wo x image
template <int DT>
inline size_t attn_wo_smem_bytes(const int hd, const int qpk, const int t_max, const int nsplit, const int q_dim,
                                 const int n_heads) {
    const size_t att = attn_smem_bytes(hd, qpk, t_max, nsplit, AW_THREADS);
    const size_t wo = LDS_HEAD_BYTES + aw_image_bytes<WDec<DT>::E>(q_dim) + sizeof(float) * (size_t)n_heads * (3 * nsplit + 1);
    return att > wo ? att : wo;
}
}  // namespace xalm
