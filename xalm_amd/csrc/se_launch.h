// se_launch.h — launchers of the stream engine (stream.h), one translation unit per weight
// dtype (se_launch.hip compiled with -DSE_DT=<id>).
#pragma once

#include <stddef.h>

#include "stream.h"

namespace xalm {

// Launch stream_decode_kernel<DT, dtc, head_dim, q per kv> on `stream`, one workgroup per CU.
// Returns 0, or an XH_E* code with a message in err[0..errlen).
#define XALM_SE_DECL(DT) \
    int se_launch_dt##DT(const SeArgs& a, int dtc, int n_cu, hipStream_t stream, char* err, size_t errlen);
XALM_SE_DECL(1)
XALM_SE_DECL(2)
XALM_SE_DECL(3)
XALM_SE_DECL(6)
XALM_SE_DECL(7)
#undef XALM_SE_DECL

inline bool se_instantiated(int hd, int qpk) { return (hd == 128 || hd == 64) && qpk == 4; }

}  // namespace xalm
