// dt_launch.hip — fused attention + Wo instantiations for one Wo dtype (-DPK_DT=<xh_dtype>).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "dt_launch.h"

#ifndef PK_DT
#error "compile with -DPK_DT=<xh_dtype id>"
#endif

namespace xalm {
namespace {

template <int DT, int HD, int QPK, bool MLP>
int aw_go(const AttnArgs& aa, const GemvArgs& ga, const GemvArgs* ma, int n_kv_heads, int t_max, unsigned* sync,
          int max_waves, hipStream_t stream, unsigned long long* trace) {
    using S = AwShape<DT>;
    constexpr int E = WDec<DT>::E;
    const int nb_wo = gemv_blocks<S>(ga.rows, max_waves / S::WAVES);
    int nb_mlp = 0;
    if constexpr (MLP) {
        using SM = AwMlpShape<DT>;
        // the fused W1/W3 role needs the Wo rows on the in-register branch (attn_wo_kernel) and
        // its own pipelined shape
        if (!aw_mlp_fits<DT>(ma->n) || ga.n != S::U * 64 * E || (ga.rows + S::ROWS - 1) / S::ROWS > nb_wo * S::WAVES)
            return XH_E_INVALID;
        nb_mlp = gemv_blocks<SM>(ma->rows, max_waves / SM::WAVES);
    }
    const size_t smem = attn_wo_smem_bytes<DT>(HD, QPK, t_max, aa.nsplit, ga.n, aa.n_heads, MLP ? ma->n : 0);
    if (smem > 160 * 1024) return XH_E_INVALID;
    auto k = attn_wo_kernel<DT, HD, QPK, MLP>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return XH_E_HIP;
        attr = true;
    }
    const int blocks = n_kv_heads * aa.nsplit + nb_wo + nb_mlp;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(AW_THREADS), smem, stream, aa, ga, n_kv_heads, sync, trace,
                       MLP ? *ma : ga, nb_wo);
    return hipGetLastError() == hipSuccess ? 0 : XH_E_HIP;
}
template <int DT, int HD, int QPK>
int aw_go2(const AttnArgs& aa, const GemvArgs& ga, const GemvArgs* ma, int n_kv_heads, int t_max, unsigned* sync,
           int max_waves, hipStream_t stream, unsigned long long* trace) {
    if (ma) return aw_go<DT, HD, QPK, true>(aa, ga, ma, n_kv_heads, t_max, sync, max_waves, stream, trace);
    return aw_go<DT, HD, QPK, false>(aa, ga, ma, n_kv_heads, t_max, sync, max_waves, stream, trace);
}

template <int DT>
int mlp_go(const GemvArgs& a13, const GemvArgs& a2, unsigned* sync, unsigned* err, hipStream_t stream,
           unsigned long long* trace) {
    if (!mlp_fits<DT>(a13.n, a2.n) || a13.rows != 2 * a2.n) return XH_E_INVALID;
    using S13 = MlpW13Shape<DT>;
    using S2 = MlpW2Shape<DT>;
    const size_t smem = mlp_smem_bytes<DT>(a13.n, a2.n);
    if (smem > 80 * 1024) return XH_E_INVALID;  // two workgroups per CU
    auto k = mlp_kernel<DT>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024) != hipSuccess)
            return XH_E_HIP;
        attr = true;
    }
    const int nb13 = gemv_blocks<S13>(a13.rows, MLP_WAVES / S13::WAVES);
    const int nb2 = gemv_blocks<S2>(a2.rows, MLP_WAVES / S2::WAVES);
    hipLaunchKernelGGL(k, dim3(nb13 + nb2), dim3(512), smem, stream, a13, a2, nb13, sync, err, trace);
    return hipGetLastError() == hipSuccess ? 0 : XH_E_HIP;
}

}  // namespace

#define XALM_CAT2(a, b) a##b
#define XALM_CAT(a, b) XALM_CAT2(a, b)
int XALM_CAT(aw_launch_dt, PK_DT)(const AttnArgs& aa, const GemvArgs& ga, const GemvArgs* ma, int head_dim, int qpk,
                                  int n_kv_heads, int t_max, unsigned* sync, int max_waves, hipStream_t stream,
                                  unsigned long long* trace) {
    if (head_dim == 128 && qpk == 4) return aw_go2<PK_DT, 128, 4>(aa, ga, ma, n_kv_heads, t_max, sync, max_waves, stream, trace);
    if (head_dim == 128 && qpk == 8) return aw_go2<PK_DT, 128, 8>(aa, ga, ma, n_kv_heads, t_max, sync, max_waves, stream, trace);
    if (head_dim == 64 && qpk == 4) return aw_go2<PK_DT, 64, 4>(aa, ga, ma, n_kv_heads, t_max, sync, max_waves, stream, trace);
    if (head_dim == 16 && qpk == 2) return aw_go2<PK_DT, 16, 2>(aa, ga, ma, n_kv_heads, t_max, sync, max_waves, stream, trace);
    return XH_E_INVALID;
}

int XALM_CAT(mlp_launch_dt, PK_DT)(const GemvArgs& a13, const GemvArgs& a2, unsigned* sync, unsigned* err,
                                   hipStream_t stream, unsigned long long* trace) {
    return mlp_go<PK_DT>(a13, a2, sync, err, stream, trace);
}

}  // namespace xalm
