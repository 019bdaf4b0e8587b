// dt_launch.hip — fused attention + Wo instantiations for one Wo dtype (-DPK_DT=<xh_dtype>).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>

#include "dt_launch.h"

#ifndef PK_DT
#error "compile with -DPK_DT=<xh_dtype id>"
#endif

namespace xalm {
namespace {

template <int DT, int HD, int QPK>
int aw_go(const AttnArgs& aa, const GemvArgs& ga, int n_kv_heads, int t_max, unsigned* sync, int max_waves,
          hipStream_t stream, unsigned long long* trace) {
    using S = AwShape<DT>;
    const size_t smem = attn_wo_smem_bytes<DT>(HD, QPK, t_max, aa.nsplit, ga.n, aa.n_heads);
    if (smem > 160 * 1024) return XH_E_INVALID;
    auto k = attn_wo_kernel<DT, HD, QPK>;
    // the LDS limit is a per-device attribute: set once for each device this process launches on
    static std::atomic<uint64_t> attr{0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return XH_E_HIP;
    if (!((attr.load() >> dev) & 1u)) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return XH_E_HIP;
        attr.fetch_or(1ull << dev);
    }
    const int blocks = n_kv_heads * aa.nsplit + gemv_blocks<S>(ga.rows, max_waves / S::WAVES);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(AW_THREADS), smem, stream, aa, ga, n_kv_heads, sync, trace);
    return hipGetLastError() == hipSuccess ? 0 : XH_E_HIP;
}

}  // namespace

#define XALM_CAT2(a, b) a##b
#define XALM_CAT(a, b) XALM_CAT2(a, b)
int XALM_CAT(aw_launch_dt, PK_DT)(const AttnArgs& aa, const GemvArgs& ga, int head_dim, int qpk, int n_kv_heads,
                                  int t_max, unsigned* sync, int max_waves, hipStream_t stream,
                                  unsigned long long* trace) {
    if (head_dim == 128 && qpk == 4) return aw_go<PK_DT, 128, 4>(aa, ga, n_kv_heads, t_max, sync, max_waves, stream, trace);
    if (head_dim == 128 && qpk == 8) return aw_go<PK_DT, 128, 8>(aa, ga, n_kv_heads, t_max, sync, max_waves, stream, trace);
    if (head_dim == 64 && qpk == 4) return aw_go<PK_DT, 64, 4>(aa, ga, n_kv_heads, t_max, sync, max_waves, stream, trace);
    if (head_dim == 16 && qpk == 2) return aw_go<PK_DT, 16, 2>(aa, ga, n_kv_heads, t_max, sync, max_waves, stream, trace);
    return XH_E_INVALID;
}

}  // namespace xalm
