// c_api.cpp — C entry points of libxalm_host.so (include/xalm_host.h).
#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/xalm_host.h"
#include "xalm.h"

namespace {
thread_local std::string g_err;

template <typename F>
int guard(F&& f) {
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return XH_E_INVALID;
    }
}
}  // namespace

extern "C" {

const char* xalm_host_last_error(void) { return g_err.c_str(); }

int xalm_read_config(const char* path, int context, xh_config* out) {
    return guard([&] { *out = xalm::Config::from_xalm(xalm::XalmFile::load(path), context).to_abi(); });
}

int xalm_encode(const char* path, const char* text, int encode_bos, int* out, int cap, int* n_out) {
    return guard([&] {
        const xalm::XalmFile f = xalm::XalmFile::load(path);
        const xalm::Tokenizer tok(f);
        const std::vector<int> ids = tok.encode(text, encode_bos != 0);
        const int n = (int)ids.size() < cap ? (int)ids.size() : cap;
        if (n > 0) memcpy(out, ids.data(), (size_t)n * sizeof(int));
        *n_out = (int)ids.size();
    });
}

int xalm_load_model(const char* path, int context, int device_ordinal, xh_ctx** out) {
    // the Model releases its context on destruction; detach it for the C caller
    return guard([&] {
        const xalm::XalmFile f = xalm::XalmFile::load(path);
        const xalm::Config c = xalm::Config::from_xalm(f, context);
        xh_config abi = c.to_abi();
        xh_ctx* ctx = nullptr;
        if (xh_create(&abi, device_ordinal, &ctx) != 0) throw std::runtime_error(xh_last_error(nullptr));
        try {
            for (const auto& kv : f.tensors) {
                const std::string& name = kv.first;
                int kind = -1, layer = 0;
                if (name == "embed.weight") kind = XH_EMBED;
                else if (name == "output.norm.weight") kind = XH_FINAL_NORM;
                else if (name == "output.weight") kind = XH_WCLS;
                else if (name.rfind("l.", 0) == 0) {
                    const size_t dot = name.find('.', 2);
                    layer = std::stoi(name.substr(2, dot - 2));
                    const std::string rest = name.substr(dot + 1);
                    static const char* names[] = {"attn.norm.weight", "mlp.norm.weight", "attn.q.weight",
                                                  "attn.k.weight", "attn.v.weight", "attn.down.weight",
                                                  "mlp.gate.weight", "mlp.down.weight", "mlp.up.weight"};
                    static const int kinds[] = {XH_ATTN_NORM, XH_FFN_NORM, XH_WQ, XH_WK, XH_WV,
                                                XH_WO, XH_W1, XH_W2, XH_W3};
                    for (int i = 0; i < 9; i++)
                        if (rest == names[i]) kind = kinds[i];
                }
                if (kind < 0) continue;  // tokenizer.tokens etc.
                if (xh_upload_file(ctx, kind, layer, kv.second.type, f.file_name.c_str(), kv.second.offset,
                                   kv.second.size) != 0)
                    throw std::runtime_error(name + ": " + xh_last_error(ctx));
            }
        } catch (...) {
            xh_destroy(ctx);
            throw;
        }
        *out = ctx;
    });
}

}  // extern "C"
