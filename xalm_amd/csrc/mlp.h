// mlp.h — the feed-forward block's two matvecs in ONE launch (XH_OPT_FUSE_MLP).
//
// Block::_block_cpu's feed-forward half (jubruckne/Xalm src/infer.cpp:455-494): rmsnorm,
// hb = act(W1 x) * (W3 x), x += W2 hb.  Same math and shapes as the two gemv launches
// (gemv<PRO_RMSNORM, EPI_GLU> then gemv<PRO_PLAIN, EPI_RESID>), with the kernel boundary between
// them replaced by an in-launch hand-off:
// * workgroups [0, nb13) run the W1/W3 matvec (the PF2P pipelined shape of the plain launch) and
//   store hb write-through; each then drains and arrives on sync[0]; the last arrival sets one
//   "hb ready" flag per XCD (sync[32 (1 + k)]);
// * workgroups [nb13, grid) own the W2 rows: each wave requests its first two weight steps, then
//   waits for its XCD's flag, stages hb with sc1 loads and streams the rest (gemv_after).
// Both roles run 8 waves per CU at once (2048 + 2048 waves, 16 per CU), so the W2 weight stream
// starts under the W1/W3 stream's tail instead of after a kernel boundary and a prologue.
// W1/W3 workgroups never wait; W2 workgroups wait only on them and come later in dispatch order,
// so progress does not depend on co-residency.  sync[] is zeroed by the layer's qkv launch
// (GemvArgs::mlp_reset) before the next use; a timeout sets the layer's sticky attn_wo word.
#pragma once

#include "gemv.h"

namespace xalm {

constexpr int MLP_SYNC_WORDS = 32 * MLP_RESET_WORDS;  // [0] W1/W3 arrivals, [32 (1 + k)] "hb ready" of XCD k
constexpr int MLP_WAVES = 2048;         // per role: 8 waves per CU each

template <int DT>
using MlpW13Shape = GemvShape<512, 2, 4, true, 4, true, 2, 2>;
// W2 rows (14336 wide for Mistral / Llama): steps of 2048 elements (4 chunks of 2-byte weights,
// 2 of one-byte), hb in 8 float4 per thread (n <= 16384)
template <int DT>
using MlpW2Shape = GemvShape<512, 2, (WDec<DT>::E >= 16 ? 2 : 4), true, 4, true, 8, 2>;

// trace (debug, null = off): per workgroup [4]: start, hand-off passed (W2) / rows done (W1/W3),
// end (after the arrival / the rows)
template <int DT>
__global__ __launch_bounds__(512, 4) void mlp_kernel(const GemvArgs a13, const GemvArgs a2, const int nb13,
                                                     unsigned* sync, unsigned* err, unsigned long long* trace) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int b = blockIdx.x;
    auto stamp = [&](const int k) {
        if (trace && threadIdx.x == 0) trace[4 * b + k] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    if (b < nb13) {
        gemv_body<DT, PRO_RMSNORM, EPI_GLU, MlpW13Shape<DT>, true>(a13, b, nb13, smem);
        stamp(1);
        arrive_publish(sync, (unsigned)nb13, sync + 32);
        stamp(2);
        return;
    }
    auto wait_hb = [&]() {
        poll_xcd_flag(sync + 32, err);
        stamp(1);
    };
    gemv_after<DT, PRO_PLAIN, EPI_RESID, MlpW2Shape<DT>>(a2, b - nb13, gridDim.x - nb13, smem, wait_hb);
    if (trace) {
        __syncthreads();
        stamp(2);
    }
}

// the fused launch takes these shapes: plain weights, W1/W3 rows in whole pipelined steps with
// x in 2 float4 per thread, W2 rows in whole steps with hb in 8 float4 per thread
template <int DT>
inline bool mlp_fits(const int dim, const int hidden) {
    using S13 = MlpW13Shape<DT>;
    using S2 = MlpW2Shape<DT>;
    constexpr int E = WDec<DT>::E;
    return WScale<DT>::BLOCK == 0 && dim % (64 * E * S13::U) == 0 && dim <= 4 * S13::XN * S13::THREADS &&
           hidden % (64 * E * S2::U) == 0 && hidden <= 4 * S2::XN * S2::THREADS;
}
template <int DT>
inline size_t mlp_smem_bytes(const int dim, const int hidden) {
    constexpr int E = WDec<DT>::E;
    auto img = [](int n) { return (size_t)((n + 64 * E - 1) / (64 * E)) * 64 * E * sizeof(float); };
    const size_t a = img(dim), b = img(hidden);
    return LDS_HEAD_BYTES + (a > b ? a : b);
}

}  // namespace xalm
