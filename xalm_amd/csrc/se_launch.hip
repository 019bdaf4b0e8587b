// se_launch.hip — stream-engine instantiations for one weight dtype (-DSE_DT=<xh_dtype>).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "se_launch.h"

#ifndef SE_DT
#error "compile with -DSE_DT=<xh_dtype id>"
#endif

namespace xalm {
namespace {

template <int DT, int DTC, int HD, int QPK>
int go(const SeArgs& a, int n_cu, hipStream_t stream, char* err, size_t errlen) {
    const size_t smem = se_smem_bytes(a.nslots, QPK, HD);
    if (smem > 160 * 1024 || a.nslots < SE_DEPTH + 1 || a.nslots > SE_MAXS) {
        snprintf(err, errlen, "stream engine: %d ring slots (%zu B of LDS) do not fit", a.nslots, smem);
        return XH_E_INVALID;
    }
    auto k = stream_decode_kernel<DT, DTC, HD, QPK>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) {
            snprintf(err, errlen, "hipFuncSetAttribute failed");
            return XH_E_HIP;
        }
        attr = true;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, SE_THREADS, smem) != hipSuccess || per_cu < 1) {
        snprintf(err, errlen, "stream kernel does not fit one workgroup per CU");
        return XH_E_INVALID;
    }
    hipLaunchKernelGGL(k, dim3(n_cu), dim3(SE_THREADS), smem, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(err, errlen, "stream launch: %s", hipGetErrorString(e));
        return XH_E_HIP;
    }
    return 0;
}

template <int DT, int DTC>
int go_hd(const SeArgs& a, int n_cu, hipStream_t stream, char* err, size_t errlen) {
    const int hd = a.head_dim, qpk = a.n_heads / a.n_kv_heads;
    if (hd == 128 && qpk == 4) return go<DT, DTC, 128, 4>(a, n_cu, stream, err, errlen);
    if (hd == 64 && qpk == 4) return go<DT, DTC, 64, 4>(a, n_cu, stream, err, errlen);
    snprintf(err, errlen, "stream engine: head_dim %d x %d q per kv not instantiated", hd, qpk);
    return XH_E_INVALID;
}

}  // namespace

#define XALM_CAT2(a, b) a##b
#define XALM_CAT(a, b) XALM_CAT2(a, b)
int XALM_CAT(se_launch_dt, SE_DT)(const SeArgs& a, int dtc, int n_cu, hipStream_t stream, char* err, size_t errlen) {
#if SE_DT == 6 || SE_DT == 7  // fp8 matrices: lm_head bf16 (convert.py) or fp8
    if (dtc == XH_BF16) return go_hd<SE_DT, XH_BF16>(a, n_cu, stream, err, errlen);
#endif
    if (dtc == SE_DT) return go_hd<SE_DT, SE_DT>(a, n_cu, stream, err, errlen);
    snprintf(err, errlen, "stream engine: unsupported dtype pair %d/%d", SE_DT, dtc);
    return XH_E_INVALID;
}

}  // namespace xalm
