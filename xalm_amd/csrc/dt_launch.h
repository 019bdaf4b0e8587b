// dt_launch.h — launchers of the big per-dtype kernel families (the persistent decode kernel,
// the fused attention + Wo kernel), one translation unit per weight dtype (dt_launch.hip
// compiled with -DPK_DT=<id>), so the instantiations build in parallel.
#pragma once

#include <stddef.h>

#include "attn_col.h"
#include "attn_wo.h"
#include "persistent.h"
#include "qaw.h"

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

// Fused attention + Wo (+ residual) launch (attn_wo.h) for Wo dtype DT: grid = the attention
// workgroups + the Wo row workgroups (at most max_waves waves).  t_max: the longest split for
// the context (attn_split_len at attn_min_t(head_dim, AW_THREADS)).  Returns 0, or XH_E_INVALID
// when (head_dim, q per kv) is not instantiated (the caller falls back to two launches).
#define XALM_AW_DECL(DT)                                                                                      \
    int aw_launch_dt##DT(const AttnArgs& aa, const GemvArgs& ga, int head_dim, int qpk, int n_kv_heads, \
                         int t_max, unsigned* sync, int max_waves, hipStream_t stream,              \
                         unsigned long long* trace);
XALM_AW_DECL(1)
XALM_AW_DECL(2)
XALM_AW_DECL(3)
XALM_AW_DECL(6)
XALM_AW_DECL(7)
XALM_AW_DECL(9)
#undef XALM_AW_DECL
// qkv + attention + Wo in one launch (qaw.h) for weight dtype DT (wq/wk/wv and Wo share it):
// grid = attention workgroups + row workgroups = 2 x n_cu.  Returns 0, or XH_E_INVALID when
// the shape is not instantiated or does not fit two workgroups per CU (caller falls back).
#define XALM_QAW_DECL(DT)                                                                                    \
    int qaw_launch_dt##DT(const GemvArgs& qa, const AttnArgs& aa, const GemvArgs& wa, int head_dim, int qpk, \
                          int n_kv_heads, int t_max, int n_cu, const QawSync& sy, hipStream_t stream);
XALM_QAW_DECL(1)
XALM_QAW_DECL(2)
XALM_QAW_DECL(3)
XALM_QAW_DECL(6)
XALM_QAW_DECL(7)
XALM_QAW_DECL(9)
#undef XALM_QAW_DECL

// Column-form attention + Wo for short histories (attn_col.h) for Wo dtype DT: grid =
// n_kv_heads x row blocks.  Returns 0, or XH_E_INVALID when the shape is not instantiated or
// a head's Wo slice is not a power-of-two number of 16-B chunks <= 64 (caller falls back).
#define XALM_AC_DECL(DT) \
    int acol_launch_dt##DT(const AttnArgs& aa, const AcArgs& ac, int head_dim, int qpk, hipStream_t stream);
XALM_AC_DECL(1)
XALM_AC_DECL(2)
XALM_AC_DECL(3)
XALM_AC_DECL(6)
XALM_AC_DECL(7)
XALM_AC_DECL(9)
#undef XALM_AC_DECL
// rows per wave of the column form (AcShape::RW), 0 = not instantiated for this dtype / shape
int acol_rows_per_wave(int dt, int head_dim, int qpk);

inline bool aw_instantiated(int hd, int qpk) {
    return (hd == 128 && (qpk == 4 || qpk == 8)) || (hd == 64 && qpk == 4) || (hd == 16 && qpk == 2);
}

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
