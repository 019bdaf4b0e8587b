/*
 * xalm_host.h — C entry points of the C++ host library (libxalm_host.so), for bindings and
 * tests.  The C++ API itself (XalmFile, Config, Model, InferenceState, Tokenizer, Sampler)
 * is in xalm_amd/host/xalm.h and mirrors jubruckne/Xalm src/model.h, src/xalm.h,
 * src/tokenizer.h, src/sampler.h.
 */
#ifndef XALM_HOST_H
#define XALM_HOST_H

#include "xalm_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Config::from_xalm (src/model.h:44-90) of a .xalm file; context 0 = cap at 4096. */
int xalm_read_config(const char* xalm_path, int context, xh_config* out);
/* Tokenizer::encode (src/tokenizer.cpp:82-119); writes at most `cap` ids, count in *n_out. */
int xalm_encode(const char* xalm_path, const char* text, int encode_bos, int* out, int cap, int* n_out);
/* Load a .xalm into a new device context (Model::from_xalm, src/model.cpp:48-118). */
int xalm_load_model(const char* xalm_path, int context, int device_ordinal, xh_ctx** out);
const char* xalm_host_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
