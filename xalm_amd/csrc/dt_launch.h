// dt_launch.h — launchers of the fused attention + Wo kernel (attn_wo.h), one translation unit
// per Wo dtype (dt_launch.hip compiled with -DPK_DT=<id>), so the instantiations build in
// parallel.
#pragma once

#include <stddef.h>

#include "attn_wo.h"

namespace xalm {

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

inline bool aw_instantiated(int hd, int qpk) {
    return (hd == 128 && (qpk == 4 || qpk == 8)) || (hd == 64 && qpk == 4) || (hd == 16 && qpk == 2);
}

}  // namespace xalm
