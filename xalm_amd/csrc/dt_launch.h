// dt_launch.h — launchers of the fused attention + Wo kernel (attn_wo.h), one translation unit
// per Wo dtype (dt_launch.hip compiled with -DPK_DT=<id>), so the instantiations build in
// parallel.
#pragma once

#include <stddef.h>

#include "attn_wo.h"
#include "mlp.h"

namespace xalm {

// Fused attention + Wo (+ residual) launch (attn_wo.h) for Wo dtype DT: grid = the attention
// workgroups + the Wo row workgroups (at most max_waves waves) [+ the W1/W3 row workgroups when
// ma != nullptr: the layer's gate/up matvec (same dtype DT) fused behind the Wo hand-off].
// t_max: the longest split for the context (attn_split_len at attn_min_t(head_dim, AW_THREADS)).
// Returns 0, or XH_E_INVALID when (head_dim, q per kv) is not instantiated or the MLP role does
// not fit the shapes (the caller falls back to separate launches).
#define XALM_AW_DECL(DT)                                                                                      \
    int aw_launch_dt##DT(const AttnArgs& aa, const GemvArgs& ga, const GemvArgs* ma, int head_dim, int qpk, \
                         int n_kv_heads, int t_max, unsigned* sync, int max_waves, hipStream_t stream,      \
                         unsigned long long* trace);
XALM_AW_DECL(1)
XALM_AW_DECL(2)
XALM_AW_DECL(3)
XALM_AW_DECL(6)
XALM_AW_DECL(7)
XALM_AW_DECL(9)
#undef XALM_AW_DECL

// W1/W3 + W2 in one launch (mlp.h) for weight dtype DT (both matrices): XH_E_INVALID when the
// shapes do not fit (the caller launches the two matvecs).  sync: the layer's MLP_SYNC_WORDS
// (zeroed), err: a sticky timeout word.
#define XALM_MLP_DECL(DT) \
    int mlp_launch_dt##DT(const GemvArgs& a13, const GemvArgs& a2, unsigned* sync, unsigned* err, hipStream_t stream, \
                          unsigned long long* trace);
XALM_MLP_DECL(1)
XALM_MLP_DECL(2)
XALM_MLP_DECL(3)
XALM_MLP_DECL(6)
XALM_MLP_DECL(7)
XALM_MLP_DECL(9)
#undef XALM_MLP_DECL

inline bool aw_instantiated(int hd, int qpk) {
    return (hd == 128 && (qpk == 4 || qpk == 8)) || (hd == 64 && qpk == 4) || (hd == 16 && qpk == 2);
}

}  // namespace xalm
