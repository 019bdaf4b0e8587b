// pk_launch.h — launchers of the persistent decode kernel, one translation unit per weight
// dtype (pk_launch.hip compiled with -DPK_DT=<id>), so the instantiations build in parallel.
#pragma once

#include <stddef.h>

#include "persistent.h"

namespace xalm {

// Launch persistent_decode_kernel<DT, dtc, head_dim, q per kv> on `stream` with one
// workgroup per CU (n_cu).  Returns 0, or an XH_E* code with a message in err[0..errlen).
#define XALM_PK_DECL(DT) \
    int pk_launch_dt##DT(const PkArgs& a, int dtc, int n_cu, hipStream_t stream, char* err, size_t errlen);
XALM_PK_DECL(1)
XALM_PK_DECL(2)
XALM_PK_DECL(3)
XALM_PK_DECL(6)
XALM_PK_DECL(7)
#undef XALM_PK_DECL

// LDS bytes one workgroup needs: the largest x image (dim, q_dim, hidden at the matrix dtype;
// dim at the lm_head dtype) or the attention tiles, behind a 512-byte header.
inline size_t pk_image_bytes(int n, int E) { return (size_t)((n + 64 * E - 1) / (64 * E)) * 64 * E * sizeof(float); }
inline size_t pk_smem_bytes(const PkArgs& a, int E, int EC, int hd, int qpk) {
    const int t_max = attn_split_len(a.max_seq_len, a.nsplit);
    size_t work = pk_image_bytes(a.dim, E);
    if (pk_image_bytes(a.q_dim, E) > work) work = pk_image_bytes(a.q_dim, E);
    if (pk_image_bytes(a.hidden, E) > work) work = pk_image_bytes(a.hidden, E);
    if (pk_image_bytes(a.dim, EC) > work) work = pk_image_bytes(a.dim, EC);
    const size_t att = sizeof(float) * ((size_t)PK_WAVES * qpk * hd + ((2 * qpk + 3) & ~3) +
                                        (size_t)qpk * (t_max > a.nsplit ? t_max : a.nsplit));
    return 512 + (att > work ? att : work);
}

}  // namespace xalm
