// attention.h — single-token GQA attention over the fp16 KV ring (split-KV "flash decoding").
//
// Replaces the head loop of Block::_block_cpu (jubruckne/Xalm src/infer.cpp:434-444) and
// `attn` (src/infer.cpp:325-359) + `softmax` (:280-297):
//   s_t = (q_h . K[t, g]) * (1/sqrtf(hd)),  t in [0, kv_len) ring slots
//   p   = softmax(s)   (max-subtract, expf)
//   o_h = sum_t p_t V[t, g],   g = h / (n_heads / n_kv_heads)
// One workgroup (16 waves) serves one KV head and a contiguous slot range, so each K/V row is
// read from HBM once for all q heads of its group (the CPU re-reads it per q head).  K and V
// rows of the first round (ATTN_PREF passes: 256 slots at hd = 128 for the short splits of the
// fused launch) are requested together at kernel start, so a short split is one HBM round trip;
// long splits stream rounds of ATTN_PREF_LONG passes with the next round in flight, with
// non-temporal loads (each row is read once per step).  The split
// length T is chosen on device from kv_len (grid shape fixed for graph replay): kv_len <= 256
// needs no merge at all.  With more than one active split, every block stores its partial
// (o, m, l) write-through and the last block of each KV head to arrive merges them (ticket
// protocol of MI355X_MICROARCH.md "Valid forms", row 1): no second launch, no fences.
#pragma once

#include <float.h>

#include <type_traits>

#include "common.h"

namespace xalm {

constexpr int ATTN_THREADS = 1024;
constexpr int ATTN_WAVES = ATTN_THREADS / 64;
// K/V passes held in registers per round (two rounds in flight).  Short splits (PARTIALS: the
// fused launch's chain at short histories) take 4 with default-policy loads: the whole split in
// the first round trip.  Long splits stream: 2 with non-temporal loads (isolated 32k split
// 31.0 -> 27.1 us; 4 / 3 passes with nt loads 28.5 / 27.8 us, tools/attn_bench), while the
// short chain measured slower with either change (4k decode -0.4 % f16, -1.3 % fp8).
constexpr int ATTN_PREF = 4;
constexpr int ATTN_PREF_LONG = 2;
constexpr int ATTN_MIN_ROUNDS = 4;  // the split floor in passes (attn_min_t)
constexpr int ATTN_MIN_T = 256;  // minimum slots per split

struct AttnArgs {
    const float* q;          // [n_heads * HD], roped
    const uint16_t* kc;      // [max_seq_len][kv_dim] fp16 bits
    const uint16_t* vc;
    int kv_dim;
    int n_heads;
    int nsplit;              // gridDim.y
    float* out;              // [n_heads * HD]
    float* part_o;           // [nsplit][n_heads][HD]
    float* part_ml;          // [nsplit][n_heads][2]
    int* counters;           // [n_kv_heads], zero between launches
    const StepParams* sp;
};

// slots per split for this step: >= min_t, multiple of 16, nsplit * T >= kv_len
__device__ __host__ __forceinline__ int attn_split_len(const int kv_len, const int nsplit,
                                                       const int min_t = ATTN_MIN_T) {
    int t = (kv_len + nsplit - 1) / nsplit;
    t = (t + 15) & ~15;
    return t < min_t ? min_t : t;
}
// one round of K/V rows per block: the split floor of a THREADS-thread block
__device__ __host__ constexpr int attn_min_t(const int hd, const int threads) { return ATTN_MIN_ROUNDS * threads / (hd / 8); }
// the fused launch's floor: half a round (each split block pulls half the bytes: a block's
// K/V fetch is bound by its CU's ~60 GB/s, so more, smaller splits shorten the chain)
__device__ __host__ constexpr int attn_min_t_partials(const int hd, const int threads) {
    return attn_min_t(hd, threads) / 2;
}

__device__ __forceinline__ float ld_sc1(const float* p) {
    return __builtin_bit_cast(float, __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(float* p, const float v) {
    __hip_atomic_store((uint32_t*)p, __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global loads (__syncthreads() drains vmcnt too, which made every wave wait for the first V
// round — a full HBM round trip — before the softmax: 2.5 us of a 32k split, tools/attn_bench)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

struct NoWait {
    __device__ void operator()() const {}
};
// PARTIALS arrival: one relaxed agent-scope add on *done (after the partial is drained)
struct AddArrive {
    __device__ void operator()(unsigned* done) const {
        __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};

// One workgroup of THREADS threads: KV head g, split s.  PARTIALS (attn_wo.h): every active
// split stores its partial (o, m, l) write-through, drains, and adds 1 to *done; the
// consumers merge (no ticket, no merge round trips inside the attention chain).
// MINT: split floor (0 = the default of the mode); `arrive(done)` runs on thread 0.
// SIGNAL (with !PARTIALS, attn_wo.h long contexts): the block that completes a KV head (its only
// split, or the last split to arrive, which merges) stores the head's output write-through,
// drains and calls arrive(done): the consumer waits for n_kv_heads arrivals and reads the
// merged output, instead of merging n_active partials itself.
template <int HD, int QPK, int THREADS, bool PARTIALS, int MINT = 0, class Wait = NoWait,
          class Arrive = AddArrive, bool SIGNAL = false>
__device__ __forceinline__ void attn_block(const AttnArgs& a, const int g, const int s, char* smem, unsigned* done,
                                           unsigned long long* dbg = nullptr, const Wait& wait = Wait(),
                                           const Arrive& arrive = Arrive()) {
#define ATTN_STAMP(k) \
    do { if (dbg && threadIdx.x == 0) dbg[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
    constexpr int WAVES = THREADS / 64;
    constexpr int PREF = PARTIALS ? ATTN_PREF : ATTN_PREF_LONG;
    constexpr int LPR = HD / 8;               // lanes per K/V row (16 B = 8 fp16 each)
    constexpr int RPP = THREADS / LPR;        // rows per pass
    constexpr int NO = QPK * HD;              // outputs of this block
    float* red = (float*)smem;                               // [WAVES][NO]
    float* ml = red + WAVES * NO;                            // [QPK][2] (+ flag)
    float* xw = ml + ((2 * QPK + 4) & ~3);                   // [2][WAVES] softmax partials of each wave
    float* sc = xw + 2 * WAVES;                              // [QPK][T]
    int* flag = (int*)(ml + 2 * QPK);

    const int kv_len = a.sp->kv_len;
    constexpr int MIN_T = MINT ? MINT : PARTIALS ? attn_min_t_partials(HD, THREADS) : ATTN_MIN_T;
    const int T = attn_split_len(kv_len, a.nsplit, MIN_T);
    const int t0 = s * T;
    if (t0 >= kv_len) return;
    const int t1 = min(kv_len, t0 + T);
    const int n_active = (kv_len + T - 1) / T;
    ATTN_STAMP(2);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int sub = tid % LPR, rr = tid / LPR;
    const float scale = 1.0f / sqrtf((float)HD);  // src/infer.cpp:338
    const size_t col = (size_t)g * HD + sub * 8;
    auto ld_kv = [&](const uint16_t* base, const int t) {
        const __attribute__((address_space(1))) u32x4* p =
            (const __attribute__((address_space(1))) u32x4*)((const char*)base + ((size_t)t * a.kv_dim + col) * 2);
        return PARTIALS ? *p : __builtin_nontemporal_load(p);
    };

    // ---- first round of K and V rows, requested before anything else ----
    u32x4 kr[PREF], vr[PREF];
#pragma unroll
    for (int p = 0; p < PREF; p++) {
        const int t = t0 + rr + p * RPP;
        if (t < t1) {
            kr[p] = ld_kv(a.kc, t);
            vr[p] = ld_kv(a.vc, t);
        }
    }
    wait();
    float qv[QPK][8];
#pragma unroll
    for (int h = 0; h < QPK; h++) {
        const size_t qo = (size_t)(g * QPK + h) * HD + sub * 8;
        const float4* qp = (const float4*)(a.q + qo);
        const float4 q0 = qp[0], q1 = qp[1];
        qv[h][0] = q0.x; qv[h][1] = q0.y; qv[h][2] = q0.z; qv[h][3] = q0.w;
        qv[h][4] = q1.x; qv[h][5] = q1.y; qv[h][6] = q1.z; qv[h][7] = q1.w;
    }

    // ---- scores ----
    auto score_row = [&](const u32x4 kw, const int t) {
        float kf[8];
        WDec<XH_F16>::dec(kw, kf);
#pragma unroll
        for (int h = 0; h < QPK; h++) {
            float p = 0.f;
#pragma unroll
            for (int i = 0; i < 8; i++) p = fmaf(qv[h][i], kf[i], p);
            p = group_reduce<LPR>(p);
            if (sub == 0) sc[h * T + (t - t0)] = p * scale;
        }
    };
    // rounds of RPP * PREF rows, software-pipelined: round r + 1 is requested before round
    // r's dot products.  Two named register sets alternate (unrolled by two): a copy of a
    // register with a load in flight would make the compiler wait for that load, and a load
    // behind a branch would merge into a vmcnt(0); the last round has its own block, so every
    // wait is counted.  (One round in flight per wave left the passes latency-bound at long
    // contexts.)
    constexpr int STEP = PREF * RPP;
    auto ld_round = [&](u32x4 (&v)[PREF], const uint16_t* base_p, const int base) {
#pragma unroll
        for (int p = 0; p < PREF; p++) v[p] = ld_kv(base_p, min(base + rr + p * RPP, t1 - 1));
    };
    auto score_round = [&](const u32x4 (&v)[PREF], const int base) {
#pragma unroll
        for (int p = 0; p < PREF; p++) {
            const int t = base + rr + p * RPP;
            if (t < t1) score_row(v[p], t);
        }
    };
    {
        u32x4 rb[PREF];
        int base = t0;
        for (;;) {
            if (base + STEP >= t1) { score_round(kr, base); break; }
            ld_round(rb, a.kc, base + STEP);
            score_round(kr, base);
            base += STEP;
            if (base + STEP >= t1) { score_round(rb, base); break; }
            ld_round(kr, a.kc, base + STEP);
            score_round(rb, base);
            base += STEP;
        }
    }
    // V round 1 is requested before the softmax (its loads do not depend on it), so the CU's
    // memory pipe is not empty across the two barriers between the K and V passes (clamped:
    // a split of one round re-reads its last row, unused)
    u32x4 vn[PREF];
    ld_round(vn, a.vc, t0 + STEP);
    lds_barrier();  // the scores are in LDS; the V loads stay in flight across the softmax
    ATTN_STAMP(3);

    // ---- softmax statistics per head (max-subtract + expf, src/infer.cpp:280-297) ----
    // WPH waves per head (all waves busy), each taking 256-score blocks: a lane holds 4
    // consecutive scores per float4, so the LDS reads and the expf of a block are independent (a
    // loop of one score per lane and iteration on one wave per head waited out an LDS round trip
    // per score: 2.4 us of a 32k split, tools/attn_bench).  The per-wave max and sum combine in
    // wave order through xw.  sc rows start 16-B aligned (T % 16 == 0); reads past len stay
    // inside the row and are masked.
    // (short splits of the fused launch keep one wave per head: no barrier between the passes)
    constexpr int WPH = PARTIALS ? 1 : (WAVES / QPK > 0 ? WAVES / QPK : 1);
    const int len = t1 - t0;
    const int sh = wid / WPH, sw = wid - sh * WPH;  // this wave's head and its share
    float* row = sc + sh * T;
    float m = -FLT_MAX;
    if (sh < QPK) {
        for (int i = 256 * sw + 4 * lane; i < len; i += 256 * WPH) {
            const float4 v = *(const float4*)(row + i);
            m = fmaxf(m, v.x);
            if (i + 1 < len) m = fmaxf(m, v.y);
            if (i + 2 < len) m = fmaxf(m, v.z);
            if (i + 3 < len) m = fmaxf(m, v.w);
        }
        m = wave_max(m);
        if (WPH > 1 && lane == 0) xw[wid] = m;
    }
    if constexpr (WPH > 1) lds_barrier();
    if (sh < QPK) {
        if constexpr (WPH > 1) {
            m = xw[sh * WPH];
#pragma unroll
            for (int k = 1; k < WPH; k++) m = fmaxf(m, xw[sh * WPH + k]);
        }
        float l = 0.f;
        for (int i = 256 * sw + 4 * lane; i < len; i += 256 * WPH) {
            const float4 v = *(const float4*)(row + i);
            float4 e;
            e.x = expf(v.x - m);
            e.y = i + 1 < len ? expf(v.y - m) : 0.f;
            e.z = i + 2 < len ? expf(v.z - m) : 0.f;
            e.w = i + 3 < len ? expf(v.w - m) : 0.f;
            *(float4*)(row + i) = e;
            l += (e.x + e.y) + (e.z + e.w);
        }
        l = wave_sum(l);
        if (lane == 0) {
            if (WPH == 1) {
                ml[2 * sh] = m;
                ml[2 * sh + 1] = l;
            } else {
                xw[WAVES + wid] = l;
            }
        }
    }
    lds_barrier();
    if constexpr (WPH > 1) {
        if (tid < QPK) {  // (m, l) per head, the waves' sums in wave order
            float mm = xw[tid * WPH], l = xw[WAVES + tid * WPH];
            for (int k = 1; k < WPH; k++) {
                mm = fmaxf(mm, xw[tid * WPH + k]);
                l += xw[WAVES + tid * WPH + k];
            }
            ml[2 * tid] = mm;
            ml[2 * tid + 1] = l;
        }
    }
    // (p . V reads only sc, complete at the barrier above; ml is read after the next barrier)
    ATTN_STAMP(6);

    // ---- p . V ----
    float acc[QPK][8];
#pragma unroll
    for (int h = 0; h < QPK; h++)
#pragma unroll
        for (int i = 0; i < 8; i++) acc[h][i] = 0.f;
    auto pv_row = [&](const u32x4 vw, const int t) {
        float vf[8];
        WDec<XH_F16>::dec(vw, vf);
#pragma unroll
        for (int h = 0; h < QPK; h++) {
            const float e = sc[h * T + (t - t0)];
#pragma unroll
            for (int i = 0; i < 8; i++) acc[h][i] = fmaf(e, vf[i], acc[h][i]);
        }
    };
    {
        auto pv_round = [&](const u32x4 (&v)[PREF], const int base) {
#pragma unroll
            for (int p = 0; p < PREF; p++) {
                const int t = base + rr + p * RPP;
                if (t < t1) pv_row(v[p], t);
            }
        };
        // round r + 1 is already in flight while round r is multiplied; round r + 2 goes into
        // round r's registers right after
        int base = t0;
        for (;;) {
            if (base + STEP >= t1) { pv_round(vr, base); break; }
            pv_round(vr, base);
            ld_round(vr, a.vc, base + 2 * STEP);
            base += STEP;
            if (base + STEP >= t1) { pv_round(vn, base); break; }
            pv_round(vn, base);
            ld_round(vn, a.vc, base + 2 * STEP);
            base += STEP;
        }
    }
    ATTN_STAMP(7);
    // reduce over the row slots of this wave (lanes sharing `sub`), then over waves (fixed order)
    if constexpr (LPR <= 16 && QPK * 8 >= 4) {
        // slots inside a 16-lane row first (DPP), then a reduce-scatter over the 4 rows: each
        // row ends with a quarter of the QPK*8 values, written by its first LPR lanes
        constexpr int N = QPK * 8;
        float v[N];
#pragma unroll
        for (int h = 0; h < QPK; h++)
#pragma unroll
            for (int i = 0; i < 8; i++) {
                float x = acc[h][i];
                if (LPR <= 1) x += dpp<DPP_ROW_ROR + 1>(x);
                if (LPR <= 2) x += dpp<DPP_ROW_ROR + 2>(x);
                if (LPR <= 4) x += dpp<DPP_ROW_ROR + 4>(x);
                if (LPR <= 8) x += dpp<DPP_ROW_ROR + 8>(x);
                v[h * 8 + i] = x;
            }
        rows_reduce_scatter<N>(v);
        const int r = lane >> 4;
        const int vb = (r & 1) * (N / 2) + (r >> 1) * (N / 4);
        if ((lane & 15) < LPR) {
#pragma unroll
            for (int k = 0; k < N / 4; k++) {
                const int vi = vb + k;
                red[wid * NO + (vi >> 3) * HD + sub * 8 + (vi & 7)] = v[k];
            }
        }
    } else {
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
    }
    __syncthreads();
    auto block_sum = [&](const int idx) {
        float o = 0.f;
#pragma unroll
        for (int w = 0; w < WAVES; w++) o += red[w * NO + idx];
        return o;
    };
    ATTN_STAMP(4);
    if (PARTIALS) {
        float* po = a.part_o + ((size_t)s * a.n_heads + g * QPK) * HD;
        for (int idx = tid; idx < NO; idx += THREADS) st_sc1(po + idx, block_sum(idx));
        if (tid < 2 * QPK) st_sc1(a.part_ml + ((size_t)s * a.n_heads + g * QPK) * 2 + tid, ml[tid]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        ATTN_STAMP(5);
        if (tid == 0) arrive(done);
        return;
    }
    auto out_st = [&](const int idx, const float v) {
        if (SIGNAL) st_sc1(a.out + (size_t)g * NO + idx, v);
        else a.out[(size_t)g * NO + idx] = v;
    };
    auto head_done = [&]() {
        if (!SIGNAL) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) arrive(done);
    };
    if (n_active == 1) {
        for (int idx = tid; idx < NO; idx += THREADS) out_st(idx, block_sum(idx) / ml[2 * (idx / HD) + 1]);
        head_done();
        return;
    }

    // ---- partial store, then the last block of this KV head merges all splits ----
    // Write-through hand-off (MI355X_MICROARCH.md, "Valid forms" table row 1): every partial
    // is stored with an agent-scope relaxed store (sc1, not kept in the non-coherent caches),
    // every storing wave drains vmcnt, one lane adds the ticket; the block whose add returns
    // n_active-1 reads every partial with agent-scope relaxed (sc1) loads.  No fences.
    float* po = a.part_o + ((size_t)s * a.n_heads + g * QPK) * HD;
    for (int idx = tid; idx < NO; idx += THREADS) st_sc1(po + idx, block_sum(idx));
    if (tid < 2 * QPK) st_sc1(a.part_ml + ((size_t)s * a.n_heads + g * QPK) * 2 + tid, ml[tid]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int ticket = __hip_atomic_fetch_add(a.counters + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = ticket == n_active - 1;
        if (last) __hip_atomic_store(a.counters + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    // merge: out = sum_s e^{m_s-M} o_s / sum_s e^{m_s-M} l_s   (per head)
    // The partials are split over MG thread groups (group k sums a contiguous range of splits,
    // left to right; the group sums are added in group order).  Every thread requests its
    // first MB partial values right behind its wave's (m, l) loads, so the (m, l) -> weights
    // step and the partial loads share one round trip.
    constexpr int MG = (THREADS / NO < WAVES - 1 ? THREADS / NO : WAVES - 1) > 0
                           ? (THREADS / NO < WAVES - 1 ? THREADS / NO : WAVES - 1) : 1;
    // partial values per thread per round trip: 4 / 8 / 16 by the group's split count (a fixed 16
    // requested clamped copies of the last split for short chunks)
#ifndef ATTN_MERGE_MB
#define ATTN_MERGE_MB 1
#endif
    float* wts = sc;        // [QPK][n_active] weights (sc is free now)
    float* den_s = red + MG * NO;  // [QPK]; red[k * NO + idx]: group sums
    const int chunk = (n_active + MG - 1) / MG;
    const int mgrp = tid / NO, midx = tid - mgrp * NO;
    const bool mact = tid < MG * NO;
    const int j0 = mgrp * chunk, j1 = min(n_active, j0 + chunk);
    const float* msrc = a.part_o + (size_t)g * NO + midx;
    const size_t mstride = (size_t)a.n_heads * HD;
    auto merge = [&](auto mb_c) {
        constexpr int MB = decltype(mb_c)::value;
        constexpr int NC = MB >= 16 ? 2 : 1;  // (m, l) loads per lane: up to 64 NC splits
        // (m, l) of head min(wid, QPK - 1), up to 2 splits per lane (n_active <= 128);
        // clamped indices so every load sits in one basic block with the partial loads
        const int h = min(wid, QPK - 1);
        float mv[2], lv[2];
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int j = min(lane + 64 * c, n_active - 1);
            const float* mlp = a.part_ml + ((size_t)j * a.n_heads + g * QPK + h) * 2;
            mv[c] = ld_sc1(mlp);
            lv[c] = ld_sc1(mlp + 1);
        }
        float pv[MB];
#pragma unroll
        for (int k = 0; k < MB; k++) pv[k] = ld_sc1(msrc + (size_t)min(j0 + k, n_active - 1) * mstride);
        if constexpr (NC == 1) { mv[1] = -FLT_MAX; lv[1] = 0.f; }
        const bool in0 = lane < n_active, in1 = NC > 1 && lane + 64 < n_active;
        const float M = wave_max(fmaxf(in0 ? mv[0] : -FLT_MAX, in1 ? mv[1] : -FLT_MAX));
        const float f0 = expf(mv[0] - M), f1 = expf(mv[1] - M);
        if (wid < QPK) {
            if (in0) wts[h * n_active + lane] = f0;
            if (in1) wts[h * n_active + lane + 64] = f1;
        }
        float den = in0 ? f0 * lv[0] : 0.f;
        den = in1 ? fmaf(f1, lv[1], den) : den;
        den = wave_sum(den);
        if (wid < QPK && lane == 0) den_s[h] = den;
        __syncthreads();
        float num = 0.f;
        if (mact) {
            const float* w = wts + (midx / HD) * n_active;
#pragma unroll
            for (int k = 0; k < MB; k++)
                if (j0 + k < j1) num = fmaf(w[j0 + k], pv[k], num);
            for (int j = j0 + MB; j < j1; j += MB) {  // further round trips (chunk > MB)
                float pw[MB];
#pragma unroll
                for (int k = 0; k < MB; k++) pw[k] = ld_sc1(msrc + (size_t)min(j + k, n_active - 1) * mstride);
#pragma unroll
                for (int k = 0; k < MB; k++)
                    if (j + k < j1) num = fmaf(w[j + k], pw[k], num);
            }
            red[mgrp * NO + midx] = num;
        }
        if constexpr (NO > THREADS) {
            // more outputs than threads (one group): the rest one by one, all splits each
            for (int idx = tid + THREADS; idx < NO; idx += THREADS) {
                const float* w = wts + (idx / HD) * n_active;
                const float* src = a.part_o + (size_t)g * NO + idx;
                float n2 = 0.f;
                for (int j = 0; j < n_active; j++) n2 = fmaf(w[j], ld_sc1(src + (size_t)j * mstride), n2);
                red[idx] = n2;
            }
        }
    };
    if (ATTN_MERGE_MB && chunk <= 4) merge(std::integral_constant<int, 4>{});
    else if (ATTN_MERGE_MB && chunk <= 8) merge(std::integral_constant<int, 8>{});
    else merge(std::integral_constant<int, 16>{});
    __syncthreads();
    for (int idx = tid; idx < NO; idx += THREADS) {
        float num = red[idx];
#pragma unroll
        for (int k = 1; k < MG; k++) num += red[k * NO + idx];
        out_st(idx, num / den_s[idx / HD]);
    }
    head_done();
}

#undef ATTN_STAMP

template <int HD, int QPK>
__global__ __launch_bounds__(ATTN_THREADS) void attn_split_kernel(const AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    attn_block<HD, QPK, ATTN_THREADS, false>(a, blockIdx.x, blockIdx.y, smem, nullptr);
}

// shared-memory bytes of attn_block<HD,QPK,threads> for a given max split length
inline size_t attn_smem_bytes(const int hd, const int qpk, const int t_max, const int nsplit,
                              const int threads = ATTN_THREADS) {
    const size_t scn = (size_t)qpk * (t_max > nsplit ? t_max : nsplit);
    return sizeof(float) * ((size_t)(threads / 64) * qpk * hd + ((2 * qpk + 4) & ~3) + 2 * (threads / 64) + scn);
}

}  // namespace xalm
