// qaw.h — the attention half of a decoder layer in ONE launch: rmsnorm + Wq/Wk/Wv (+ clip,
// rope, fp16 KV write), attention over the ring, Wo (+ residual).
//
// Same math as gemv_kernel<PRO_RMSNORM, EPI_QKV> -> attn_wo_kernel (jubruckne/Xalm
// src/infer.cpp:380-452), with both launch boundaries replaced by in-launch hand-offs, so the
// qkv weight stream, the K/V history reads and the Wo weight stream overlap:
// * workgroups [0, natt) are attention workgroups (KV head g = b / nsplit, split s): they
//   request their first round of K/V history rows at once, then wait for the qkv phase
//   (attention.h FUSED: the rows this launch writes and q are read after the hand-off, sc1);
//   inactive splits (past kv_len) arrive at once;
// * workgroups [natt, grid) are "row" workgroups: each wave computes its qkv row groups
//   (PF prologue: x and the attention norm in registers, first weight chunks in flight),
//   stores q / K / V write-through, and the workgroup arrives on its XCD shard of the qkv
//   counter; then each wave requests its whole Wo row group (and the residual), waits for
//   every attention workgroup, merges the split partials into the Wo input image (sc1 loads)
//   and finishes x += Wo . attn.
// Hand-offs: MI355X_MICROARCH.md "Valid forms" row 1 (sc1 stores, every storing wave drained,
// one add per workgroup; one polling lane per workgroup with relaxed sc1 loads + s_sleep).
// Counters are monotonic: targets are epoch x arrivals (epoch = forward steps since reset,
// advanced by embed_kernel), so nothing is reset between launches.  Residency: grid <= 2 x CUs
// of 512-thread workgroups at <= 128 VGPRs and <= 80 KiB LDS (host-checked), so every
// workgroup is resident and no wait depends on dispatch order.  Every spin is bounded (2 s,
// then the sticky error word is set and the launch drains).
#pragma once

#include "attn_wo.h"
#include "chain.h"

namespace xalm {

constexpr int QAW_THREADS = 512;
constexpr int QAW_WAVES = QAW_THREADS / 64;
// qkv rows: PF prologue (x of n <= 4096 in 2 float4 per thread), 2 rows x 4 chunks per wave
template <int DT>
using QawQkvShape = GemvShape<QAW_THREADS, 2, 4, true, 4, true, 2>;
// Wo rows: one group per wave, the whole row in flight (f16/bf16 4096: 8 chunks; fp8: 4)
template <int DT>
using QawWoShape = GemvShape<QAW_THREADS, 2, (WDec<DT>::E >= 16 ? 4 : 8), true, 4, false>;

// attention split floor: one full round of K/V rows per workgroup (128 slots at head_dim
// 128), so a 4k-context decode has at most ceil(kv_len / 128) partials to merge
template <int HD>
__host__ __device__ constexpr int qaw_min_t() { return attn_min_t(HD, QAW_THREADS); }

// counters of one layer, each on its own 128-B line
struct QawSync {
    unsigned* qkv;     // [CHAIN_SHARDS * CHAIN_SHARD_STRIDE] qkv-phase arrivals (row workgroups)
    unsigned* heads;   // [1] attention-workgroup arrivals, then [CHAIN_SHARDS] per-XCD "heads
                       // done" flags (= epoch), set by the last arriving attention workgroup
    const unsigned* epoch;  // forward steps since reset (embed_kernel advances it)
    int* err;          // sticky timeout word
    unsigned long long* trace;  // debug (null = off): per workgroup [8] s_memrealtime stamps
};

__device__ __forceinline__ bool qaw_poll(const unsigned* c, const int shards, const unsigned target, int* err) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        unsigned s = 0;
        for (int k = 0; k < shards; k++) s += ld_sc1_u32(c + k * CHAIN_SHARD_STRIDE);
        if (s >= target) return true;
        if (ld_sc1_u32(err)) return false;
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
            st_sc1_u32(err, 1u);
            return false;
        }
    }
}

// K[r] = f16(rope(f32(K[r]), pos = 1)) for the sink rows (src/infer.cpp:421-431), write-through
template <int THREADS>
__device__ __forceinline__ void rotate_sinks_sc1(const GemvArgs& a, const int kv_sink) {
    for (int r = 0; r < kv_sink; r++) {
        uint16_t* krow = a.kcache + (size_t)r * a.kv_dim;
        for (int p = threadIdx.x; p < (a.kv_dim >> 1); p += THREADS) {
            const int i = p << 1;
            const int jh = (i % a.head_dim) >> 1;
            const uint32_t kk = ld_sc1_u32(krow + i);
            const float k0 = f16_bits_to_f32((uint16_t)kk), k1 = f16_bits_to_f32((uint16_t)(kk >> 16));
            const float fcr = a.sink_cos[jh], fci = a.sink_sin[jh];
            st_sc1_u32(krow + i, (uint32_t)f32_to_f16_bits(k0 * fcr - k1 * fci) |
                                     ((uint32_t)f32_to_f16_bits(k0 * fci + k1 * fcr) << 16));
        }
    }
}

template <int DT, int HD, int QPK>
__global__ __launch_bounds__(QAW_THREADS, 4) void qkv_attn_wo_kernel(const GemvArgs qa, const AttnArgs aa,
                                                                     const GemvArgs wa, const int n_kv_heads,
                                                                     const QawSync sy) {
    constexpr int E = WDec<DT>::E;
    using SQ = QawQkvShape<DT>;
    using SW = QawWoShape<DT>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int natt = n_kv_heads * aa.nsplit;
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned epoch = *sy.epoch;  // written by embed_kernel in an earlier launch
    const int n_rowb = gridDim.x - natt;
    // trace: [0] start; attention: [1] hand-off passed (via wait), [2..7] attn_block's stamps;
    // rows: [1] qkv staged, [2] qkv arrived, [3] heads passed, [4] merged, [5] end
    unsigned long long* tr = sy.trace ? sy.trace + 8 * b : nullptr;
#define QAW_STAMP(k) \
    do { if (tr && threadIdx.x == 0) tr[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
    QAW_STAMP(0);

    if (b < natt) {
        // ---- attention workgroup ----
        const int g = b / aa.nsplit, s = b - g * aa.nsplit;
        auto wait_qkv = [&]() {
            if (threadIdx.x == 0) qaw_poll(sy.qkv, CHAIN_SHARDS, epoch * (unsigned)n_rowb, sy.err);
            __syncthreads();
            QAW_STAMP(1);
        };
        // arrival; the last of the natt arrivals of this epoch sets the per-XCD flags (one
        // polled line per XCD instead of every row workgroup on one counter)
        auto arrive = [&](unsigned* c) {
            const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1 == epoch * (unsigned)natt) {
#pragma unroll
                for (int k = 0; k < CHAIN_SHARDS; k++) st_sc1_u32(c + (1 + k) * CHAIN_SHARD_STRIDE, epoch);
            }
        };
        const int kv_len = aa.sp->kv_len;
        const int T = attn_split_len(kv_len, aa.nsplit, qaw_min_t<HD>());
        if (s * T < kv_len) {
            // publishes its partial write-through and arrives on sy.heads
            attn_block<HD, QPK, QAW_THREADS, true, true, qaw_min_t<HD>()>(aa, g, s, smem, sy.heads, tr, wait_qkv,
                                                                          arrive);
        } else if (threadIdx.x == 0) {
            arrive(sy.heads);
        }
        return;
    }

    // ---- row workgroup: qkv rows ----
    const int rb = b - natt;
    {
        float* red = (float*)smem;
        float4* xs4 = (float4*)(smem + LDS_HEAD_BYTES);
        const int g = rb * QAW_WAVES + wid;
        const int n_groups = gemv_groups<SQ>(qa);
        const int total = n_rowb * QAW_WAVES;
        // PF prologue when the shape allows it (uniform), else the plain one
        if (qa.n >= 64 * E * SQ::U && qa.n <= 4 * SQ::XN * QAW_THREADS) {
            float4 xv[SQ::XN], nw[SQ::XN];
            stage_x_issue<PRO_RMSNORM, SQ>(qa, xv, nw);
            u32x4 pre[SQ::U][SQ::ROWS];
            gemv_prefetch<SQ>(qa, min(g, n_groups - 1), lane, pre);
            stage_x_finish<E, PRO_RMSNORM, SQ>(qa, xv, nw, xs4, red);
            if (rb == 0) rotate_sinks_sc1<QAW_THREADS>(qa, qa.sp->kv_sink);
            __syncthreads();
            QAW_STAMP(1);
            if (g < n_groups) gemv_rows<DT, EPI_QKV, SQ, true, true>(qa, g, total, lane, xs4, pre);
        } else {
            stage_x<E, PRO_RMSNORM, QAW_THREADS>(qa, xs4, red);
            if (rb == 0) rotate_sinks_sc1<QAW_THREADS>(qa, qa.sp->kv_sink);
            __syncthreads();
            u32x4 none[SQ::U][SQ::ROWS];
            gemv_rows<DT, EPI_QKV, SQ, false, true>(qa, g, total, lane, xs4, none);
        }
        // qkv outputs drained, one arrival per workgroup on this XCD's shard
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_fetch_add(sy.qkv + xcc_id() * CHAIN_SHARD_STRIDE, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        QAW_STAMP(2);
    }

    // ---- row workgroup: Wo rows (+ residual) ----
    const int gw = rb * QAW_WAVES + wid;
    const int nw_groups = gemv_groups<SW>(wa);
    // any Wo rows in this workgroup?  (uniform; idle workgroups leave without waiting)
    if (rb * QAW_WAVES >= nw_groups) return;
    const int kv_len = aa.sp->kv_len;
    const int T = attn_split_len(kv_len, aa.nsplit, qaw_min_t<HD>());
    const int n_active = (kv_len + T - 1) / T;
    float4* xs4 = (float4*)(smem + LDS_HEAD_BYTES);
    float* wts = (float*)(smem + LDS_HEAD_BYTES + aw_image_bytes<E>(wa.n));
    auto wait_heads = [&]() {
        if (threadIdx.x == 0) qaw_poll(sy.heads + (1 + xcc_id()) * CHAIN_SHARD_STRIDE, 1, epoch, sy.err);
        __syncthreads();
        QAW_STAMP(3);
        aw_stage_merged<E, HD, QAW_THREADS>(aa, wa.n, n_active, xs4, wts);
        __syncthreads();
        QAW_STAMP(4);
    };
    if (wa.n == SW::U * 64 * E && nw_groups <= n_rowb * QAW_WAVES) {
        // at most one group per wave, whole rows in the U chunks: request them (and the
        // residual), then wait
        const bool has_wo = gw < nw_groups;
        u32x4 w[SW::U][SW::ROWS];
        float xres[SW::ROWS];
        if (has_wo) {
            gemv_prefetch<SW>(wa, gw, lane, w);
            if (lane == 0) {
#pragma unroll
                for (int r = 0; r < SW::ROWS; r++) xres[r] = gw * SW::ROWS + r < wa.rows ? wa.out[gw * SW::ROWS + r] : 0.f;
            }
        }
        wait_heads();
        if (has_wo) {
            float acc[SW::ROWS];
#pragma unroll
            for (int r = 0; r < SW::ROWS; r++) acc[r] = 0.f;
            gemv_compute<DT, SW::ROWS, SW::U>(w, xs4, 0, lane, acc);
#pragma unroll
            for (int r = 0; r < SW::ROWS; r++) acc[r] = wave_sum(acc[r]);
            if (lane == 0) {
#pragma unroll
                for (int r = 0; r < SW::ROWS; r++)  // x += Wo . attn (src/infer.cpp:449-452)
                    if (gw * SW::ROWS + r < wa.rows) wa.out[gw * SW::ROWS + r] = xres[r] + acc[r];
            }
        }
    } else {
        wait_heads();
        using G = GemvShape<QAW_THREADS, 2, 4, true, 4, false>;
        u32x4 none[G::U][G::ROWS];
        gemv_rows<DT, EPI_RESID, G, false>(wa, gw, n_rowb * QAW_WAVES, lane, xs4, none);
    }
    if (tr) {
        __syncthreads();
        QAW_STAMP(5);
    }
#undef QAW_STAMP
}

// LDS bytes of one workgroup: the attention tiles or the row-workgroup images
template <int DT>
inline size_t qaw_smem_bytes(const int hd, const int qpk, const int t_max, const int nsplit, const int dim,
                             const int q_dim, const int n_heads) {
    constexpr int E = WDec<DT>::E;
    const size_t att = attn_smem_bytes(hd, qpk, t_max, nsplit, QAW_THREADS);
    const size_t qkv = LDS_HEAD_BYTES + aw_image_bytes<E>(dim);
    const size_t wo = LDS_HEAD_BYTES + aw_image_bytes<E>(q_dim) + sizeof(float) * (size_t)n_heads * (3 * nsplit + 1);
    size_t m = att > qkv ? att : qkv;
    return m > wo ? m : wo;
}

}  // namespace xalm
