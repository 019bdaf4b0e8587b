// dt_launch.hip — persistent-kernel and fused attention + Wo instantiations for one weight
// dtype (-DPK_DT=<xh_dtype>).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "dt_launch.h"

#ifndef PK_DT
#error "compile with -DPK_DT=<xh_dtype id>"
#endif

namespace xalm {
namespace {

template <int DT, int DTC, int HD, int QPK>
int go(const PkArgs& a, int n_cu, hipStream_t stream, char* err, size_t errlen) {
    const size_t smem = pk_smem_bytes(a, WDec<DT>::E, WDec<DTC>::E, HD, QPK);
    if (smem > 160 * 1024) {
        snprintf(err, errlen, "persistent kernel LDS %zu B exceeds 160 KiB", smem);
        return XH_E_INVALID;
    }
    auto k = persistent_decode_kernel<DT, DTC, HD, QPK>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) {
            snprintf(err, errlen, "hipFuncSetAttribute failed");
            return XH_E_HIP;
        }
        attr = true;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, PK_THREADS, smem) != hipSuccess || per_cu < 1) {
        snprintf(err, errlen, "persistent kernel does not fit one workgroup per CU");
        return XH_E_INVALID;
    }
    hipLaunchKernelGGL(k, dim3(n_cu), dim3(PK_THREADS), smem, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(err, errlen, "persistent launch: %s", hipGetErrorString(e));
        return XH_E_HIP;
    }
    return 0;
}

template <int DT, int DTC>
int go_hd(const PkArgs& a, int n_cu, hipStream_t stream, char* err, size_t errlen) {
    const int hd = a.head_dim, qpk = a.n_heads / a.n_kv_heads;
    if (hd == 128 && qpk == 4) return go<DT, DTC, 128, 4>(a, n_cu, stream, err, errlen);
    if (hd == 128 && qpk == 8) return go<DT, DTC, 128, 8>(a, n_cu, stream, err, errlen);
    if (hd == 64 && qpk == 4) return go<DT, DTC, 64, 4>(a, n_cu, stream, err, errlen);
    if (hd == 16 && qpk == 2) return go<DT, DTC, 16, 2>(a, n_cu, stream, err, errlen);
    snprintf(err, errlen, "persistent engine: head_dim %d x %d q per kv not instantiated", hd, qpk);
    return XH_E_INVALID;
}

int unsupported(int dt, int dtc, char* err, size_t errlen) {
    snprintf(err, errlen, "persistent engine: unsupported dtype pair %d/%d", dt, dtc);
    return XH_E_INVALID;
}

template <int DT, int HD, int QPK>
int aw_go(const AttnArgs& aa, const GemvArgs& ga, int n_kv_heads, int t_max, unsigned* sync, int max_waves,
          hipStream_t stream, unsigned long long* trace) {
    using S = AwShape<DT>;
    const size_t smem = attn_wo_smem_bytes<DT>(HD, QPK, t_max, aa.nsplit, ga.n, aa.n_heads);
    if (smem > 160 * 1024) return XH_E_INVALID;
    auto k = attn_wo_kernel<DT, HD, QPK>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return XH_E_HIP;
        attr = true;
    }
    const int blocks = n_kv_heads * aa.nsplit + gemv_blocks<S>(ga.rows, max_waves / S::WAVES);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(AW_THREADS), smem, stream, aa, ga, n_kv_heads, sync, trace);
    return hipGetLastError() == hipSuccess ? 0 : XH_E_HIP;
}

template <int DT, int HD, int QPK>
int qaw_go(const GemvArgs& qa, const AttnArgs& aa, const GemvArgs& wa, int n_kv_heads, int t_max, int n_cu,
           const QawSync& sy, hipStream_t stream) {
    const size_t smem = qaw_smem_bytes<DT>(HD, QPK, t_max, aa.nsplit, qa.n, wa.n, aa.n_heads);
    if (smem > 80 * 1024) return XH_E_INVALID;  // two workgroups per CU
    auto k = qkv_attn_wo_kernel<DT, HD, QPK>;
    static int per_cu = -1;
    if (per_cu < 0) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024) != hipSuccess)
            return XH_E_HIP;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, QAW_THREADS, 80 * 1024) != hipSuccess) per_cu = 0;
    }
    if (per_cu < 2) return XH_E_INVALID;
    const int grid = 2 * n_cu;
    if (n_kv_heads * aa.nsplit >= grid) return XH_E_INVALID;
    hipLaunchKernelGGL(k, dim3(grid), dim3(QAW_THREADS), smem, stream, qa, aa, wa, n_kv_heads, sy);
    return hipGetLastError() == hipSuccess ? 0 : XH_E_HIP;
}

template <int DT, int HD, int QPK>
int acol_go(const AttnArgs& aa, const AcArgs& ac, hipStream_t stream) {
    using SH = AcShape<DT, HD, QPK>;
    if constexpr (!SH::OK) {
        return XH_E_INVALID;
    } else {
        if (ac.rows_per_wave != SH::RW) return XH_E_INVALID;
        constexpr size_t smem = attn_wo_col_smem_bytes<HD, QPK>();
        static_assert(smem <= 160 * 1024, "column-form LDS");
        auto k = attn_wo_col_kernel<DT, HD, QPK>;
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
                return XH_E_HIP;
            attr = true;
        }
        const int rb = (ac.dim + SH::ROWS - 1) / SH::ROWS;
        hipLaunchKernelGGL(k, dim3(rb * ac.n_kv_heads), dim3(AC_THREADS), smem, stream, aa, ac);
        return hipGetLastError() == hipSuccess ? 0 : XH_E_HIP;
    }
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

int XALM_CAT(qaw_launch_dt, PK_DT)(const GemvArgs& qa, const AttnArgs& aa, const GemvArgs& wa, int head_dim,
                                   int qpk, int n_kv_heads, int t_max, int n_cu, const QawSync& sy,
                                   hipStream_t stream) {
    if (head_dim == 128 && qpk == 4) return qaw_go<PK_DT, 128, 4>(qa, aa, wa, n_kv_heads, t_max, n_cu, sy, stream);
    if (head_dim == 128 && qpk == 8) return qaw_go<PK_DT, 128, 8>(qa, aa, wa, n_kv_heads, t_max, n_cu, sy, stream);
    if (head_dim == 64 && qpk == 4) return qaw_go<PK_DT, 64, 4>(qa, aa, wa, n_kv_heads, t_max, n_cu, sy, stream);
    if (head_dim == 16 && qpk == 2) return qaw_go<PK_DT, 16, 2>(qa, aa, wa, n_kv_heads, t_max, n_cu, sy, stream);
    return XH_E_INVALID;
}

int XALM_CAT(acol_launch_dt, PK_DT)(const AttnArgs& aa, const AcArgs& ac, int head_dim, int qpk, hipStream_t stream) {
    if (head_dim == 128 && qpk == 4) return acol_go<PK_DT, 128, 4>(aa, ac, stream);
    if (head_dim == 128 && qpk == 8) return acol_go<PK_DT, 128, 8>(aa, ac, stream);
    if (head_dim == 64 && qpk == 4) return acol_go<PK_DT, 64, 4>(aa, ac, stream);
    if (head_dim == 16 && qpk == 2) return acol_go<PK_DT, 16, 2>(aa, ac, stream);
    return XH_E_INVALID;
}

#if PK_DT == 2  // one definition: the shape table is dtype-generic
namespace {
template <int DT>
int rw_of(int hd, int qpk) {
    if (hd == 128 && qpk == 4) return AcShape<DT, 128, 4>::OK ? AcShape<DT, 128, 4>::RW : 0;
    if (hd == 128 && qpk == 8) return AcShape<DT, 128, 8>::OK ? AcShape<DT, 128, 8>::RW : 0;
    if (hd == 64 && qpk == 4) return AcShape<DT, 64, 4>::OK ? AcShape<DT, 64, 4>::RW : 0;
    if (hd == 16 && qpk == 2) return AcShape<DT, 16, 2>::OK ? AcShape<DT, 16, 2>::RW : 0;
    return 0;
}
}  // namespace
int acol_rows_per_wave(int dt, int head_dim, int qpk) {
    switch (dt) {
        case XH_F32: return rw_of<XH_F32>(head_dim, qpk);
        case XH_F16: return rw_of<XH_F16>(head_dim, qpk);
        case XH_BF16: return rw_of<XH_BF16>(head_dim, qpk);
        case XH_F8_E4M3: return rw_of<XH_F8_E4M3>(head_dim, qpk);
        case XH_F8_E5M2: return rw_of<XH_F8_E5M2>(head_dim, qpk);
        case XH_Q8: return rw_of<XH_Q8>(head_dim, qpk);
        default: return 0;
    }
}
#endif

#if PK_DT != 9  // no persistent engine for Q8
int XALM_CAT(pk_launch_dt, PK_DT)(const PkArgs& a, int dtc, int n_cu, hipStream_t stream, char* err, size_t errlen) {
#if PK_DT == 6 || PK_DT == 7  // fp8 matrices: lm_head bf16 (convert.py) or fp8
    if (dtc == XH_BF16) return go_hd<PK_DT, XH_BF16>(a, n_cu, stream, err, errlen);
#endif
    if (dtc == PK_DT) return go_hd<PK_DT, PK_DT>(a, n_cu, stream, err, errlen);
    return unsupported(PK_DT, dtc, err, errlen);
}
#endif

}  // namespace xalm
