// chain.h — overlapped launch chain: consecutive decode kernels run on two alternating HIP
// streams, so kernel k+1 is resident while kernel k still streams its weights.
//
// Batch-1 decode is a strict chain (qkv -> attention/Wo -> W1/W3 -> W2 -> next layer), and on
// one stream every launch pays a ramp: dispatch, the x prologue and the first HBM round trip
// (≈2-4 µs on a 8-50 µs kernel, measured per kernel in profiles/r01_gemv_bench.txt).  Here the
// weight stream of kernel k+1 does not wait for kernel k: its workgroups are dispatched as soon
// as the other stream is free, request their first weight chunks into registers, and only then
// wait for kernel k's completion count.  The dependency is carried by an in-launch style
// hand-off (MI355X_MICROARCH.md "Valid forms", row 1):
//   producer: activations stored write-through (sc1) -> every storing wave `s_waitcnt vmcnt(0)`
//             -> workgroup barrier -> one lane adds 1 to its shard of the completion counter;
//   consumer: one lane polls the 8 shards with relaxed (sc1) loads until they sum to the
//             producer's grid, workgroup barrier, then every load of the handed-off bytes is an
//             sc1 load.
// Residency (no deadlock): each chain kernel is at most one 512-thread workgroup per CU at
// <= 128 VGPRs and <= 80 KB LDS, so kernel k and k+1 (one per stream; a stream runs its kernels
// in order, so k+2 starts only after k has ended) always fit together.  Every spin is bounded
// (2 s, then the sticky error word is set and the kernel drains).
//
// Within a workgroup, wave 0 polls and stages the x image while waves 1.. hold their
// prefetched weight chunks: a wave's loads complete in issue order for `s_waitcnt vmcnt`, so a
// wave with weights in flight cannot read x without first waiting for the weights.
#pragma once

#include "gemv.h"

namespace xalm {

constexpr int CHAIN_SHARDS = 8;        // completion-counter shards (one per XCD)
constexpr int CHAIN_SHARD_STRIDE = 32;  // uints between shards (own 128-B line)
constexpr int CHAIN_SLOT = CHAIN_SHARDS * CHAIN_SHARD_STRIDE;  // uints per counter

struct ChainSync {
    unsigned* wait;    // counter of the kernel this one depends on (null: none)
    unsigned target;   // its completion count (producer workgroups)
    unsigned* sig;     // this kernel's counter (null: none)
    int* err;          // sticky timeout word
    unsigned long long* trace;  // debug (null = off): per workgroup [4] start, x staged, rows done, signalled
};

__device__ __forceinline__ uint32_t chain_ld(const void* p) { return ld_sc1_u32(p); }
__device__ __forceinline__ void chain_st(void* p, const uint32_t v) { st_sc1_u32(p, v); }

__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 3)" : "=s"(v));
    return v & 7;
}

// thread 0: poll until the producer's shards sum to target (bounded); caller barriers after
__device__ __forceinline__ void chain_poll(const ChainSync& sy) {
    if (!sy.wait) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        unsigned s = 0;
#pragma unroll
        for (int k = 0; k < CHAIN_SHARDS; k++) s += chain_ld(sy.wait + k * CHAIN_SHARD_STRIDE);
        if (s >= sy.target) break;
        if (chain_ld(sy.err)) break;
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
            chain_st(sy.err, 1u);
            break;
        }
    }
}

// every wave's activation stores drained, then one add to this XCD's shard
__device__ __forceinline__ void chain_signal(const ChainSync& sy) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && sy.sig)
        __hip_atomic_fetch_add(sy.sig + xcc_id() * CHAIN_SHARD_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// x image by ONE wave (sc1 loads), rms-normalised for PRO_RMSNORM; 8 float4 per lane in
// flight.  Same permuted layout as stage_x; same rms value as block_rms_scale up to the
// summation order.
template <int E, int PRO>
__device__ __forceinline__ void chain_stage_wave(const GemvArgs& a, float4* xs4, const int lane) {
    const int n4 = a.n >> 2;
    float ss = 0.f;
    auto put = [&](const int i, const float4 v) {
        const int c = i << 2;
        const int it = c / (64 * E);
        const int rem = c - it * 64 * E;
        const int l = rem / E;
        const int qd = (rem - l * E) >> 2;
        xs4[(it * (E / 4) + qd) * 64 + l] = v;
    };
    constexpr int B = 4;
    int i0 = 0;
    for (; i0 + 64 * B <= n4; i0 += 64 * B) {
        u32x4 u[B];
#pragma unroll
        for (int j = 0; j < B; j++) u[j] = ld_sc1_x4(a.x, (uint32_t)(i0 + j * 64 + lane) * 16);
#pragma unroll
        for (int j = 0; j < B; j++) {
            const float4 v = make_float4(bits_f32(u[j].x), bits_f32(u[j].y), bits_f32(u[j].z), bits_f32(u[j].w));
            ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
            put(i0 + j * 64 + lane, v);
        }
    }
    for (int i = i0 + lane; i < n4; i += 64) {
        const u32x4 u = ld_sc1_x4(a.x, (uint32_t)i * 16);
        const float4 v = make_float4(bits_f32(u.x), bits_f32(u.y), bits_f32(u.z), bits_f32(u.w));
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        put(i, v);
    }
    if (PRO == PRO_RMSNORM) {
        ss = wave_sum(ss);
        const float scale = 1.0f / sqrtf(ss / (float)a.n + a.eps);
        for (int i = lane; i < n4; i += 64) {
            const int c = i << 2;
            const int it = c / (64 * E);
            const int rem = c - it * 64 * E;
            const int l = rem / E;
            const int qd = (rem - l * E) >> 2;
            float4& v = xs4[(it * (E / 4) + qd) * 64 + l];
            const float4 w = load_norm4(a.norm_w, a.norm_dtype, i);
            v.x = v.x * scale * w.x;  // x[i] * scale * weight[i], src/infer.cpp:234
            v.y = v.y * scale * w.y;
            v.z = v.z * scale * w.z;
            v.w = v.w * scale * w.w;
        }
    }
}

// One chain gemv: waves 1.. request their first group's first U chunks, wave 0 waits for the
// producer and stages x, then every wave streams its groups (as gemv_kernel).
template <int DT, int PRO, int EPI, class S>
__global__ __launch_bounds__(S::THREADS, S::MINW) void chain_gemv_kernel(const GemvArgs a, const ChainSync sy) {
    constexpr int E = WDec<DT>::E;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float4* xs4 = (float4*)(smem + LDS_HEAD_BYTES);
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int g = blockIdx.x * S::WAVES + wid;
    if (sy.trace && threadIdx.x == 0) sy.trace[4 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    if (wid != 0) {
        // streaming waves: first chunks in flight, then wait for the staged x
        const bool prefetched = g < gemv_groups<S>(a) && a.n / (64 * E) >= S::U;
        u32x4 pre[S::U][S::ROWS];
        if (prefetched) gemv_prefetch<S>(a, g, lane, pre);
        __syncthreads();
        if (prefetched) gemv_rows<DT, EPI, S, true, true>(a, g, gridDim.x * S::WAVES, lane, xs4, pre);
        else gemv_rows<DT, EPI, S, false, true>(a, g, gridDim.x * S::WAVES, lane, xs4, pre);
    } else {
        if (lane == 0) chain_poll(sy);
        // lane 0's poll ends before the wave goes on: the staging loads follow the hand-off
        chain_stage_wave<E, PRO>(a, xs4, lane);
        if (EPI == EPI_QKV && blockIdx.x == 0) {
            // sink re-rotation (src/infer.cpp:421-431), rows 0..kv_sink-1, by wave 0 of block 0
            const int kv_sink = a.sp->kv_sink;
            for (int r = 0; r < kv_sink; r++) {
                uint16_t* krow = a.kcache + (size_t)r * a.kv_dim;
                for (int p = lane; p < (a.kv_dim >> 1); p += 64) {
                    const int i = p << 1;
                    const int jh = (i % a.head_dim) >> 1;
                    const uint32_t kk = chain_ld(krow + i);
                    const float k0 = f16_bits_to_f32((uint16_t)kk), k1 = f16_bits_to_f32((uint16_t)(kk >> 16));
                    const float fcr = a.sink_cos[jh], fci = a.sink_sin[jh];
                    chain_st(krow + i, (uint32_t)f32_to_f16_bits(k0 * fcr - k1 * fci) |
                                           ((uint32_t)f32_to_f16_bits(k0 * fci + k1 * fcr) << 16));
                }
            }
        }
        if (sy.trace && lane == 0) sy.trace[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        __syncthreads();
        u32x4 none[S::U][S::ROWS];
        gemv_rows<DT, EPI, S, false, true>(a, g, gridDim.x * S::WAVES, lane, xs4, none);
    }
    if (sy.trace) {
        __syncthreads();
        if (threadIdx.x == 0) sy.trace[4 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime();
    }
    chain_signal(sy);
    if (sy.trace && threadIdx.x == 0) sy.trace[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace xalm
