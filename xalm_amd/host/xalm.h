// xalm.h — C++ host mirror of the reference API this path plugs into (jubruckne/Xalm):
//
//   Xalm::load / file_info / tensor_info      src/xalm.h:11-192
//   Config::from_xalm                         src/model.h:25-91
//   InferenceState                            src/model.h:96-156   (host logits only)
//   InferenceMode                             src/model.h:249-252
//   Device + Model::from_xalm / forward       src/model.h:21-23, 254-284; src/model.cpp:48-122
//   Model::active_bytes                       src/model.cpp:12-35
//   Tokenizer                                 src/tokenizer.h/.cpp
//   Sampler                                   src/sampler.h/.cpp
//
// Model::forward goes through the C ABI of libxalm_hip.so (include/xalm_hip.h); Device::HIP
// is the MI355X path.  Device::CPU is the reference's own CPU forward, which this product does
// not ship (its restatement lives in oracle/ as the test checker), so selecting it throws.
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/xalm_hip.h"

namespace xalm {

// ---- .xalm container ------------------------------------------------------------------
struct TensorInfo {
    std::string name;
    int type = 0;              // enum xh_dtype
    std::vector<int> shape;
    size_t offset = 0;         // absolute file offset
    size_t size = 0;           // bytes
};

struct XalmFile {
    std::string file_name;
    std::string arch;
    std::map<std::string, std::string> metadata;  // config values (strings, convert.py:223-245)
    std::map<std::string, TensorInfo> tensors;

    static XalmFile load(const std::string& path);  // Xalm::load, src/xalm.h:90-192
    void read(const TensorInfo& ti, void* dst) const;
    std::vector<uint8_t> read(const std::string& name) const;
    const std::string& meta(const std::string& key) const;
    std::string meta_or(const std::string& key, const std::string& dflt) const;
};

int parse_type(const std::string& s);  // Type::parse, src/types.h:468-499
size_t type_size(int type);

// ---- model ------------------------------------------------------------------------------
enum class Device { CPU, HIP };
enum class InferenceMode { HYDRATE_KV_CACHE = XH_HYDRATE_KV_CACHE, OUTPUT_LOGITS = XH_OUTPUT_LOGITS };
enum class ActivationType { GELU = XH_ACT_GELU, SILU = XH_ACT_SILU };

struct Config {
    int dim = 0, hidden_dim = 0, head_dim = 0, n_layers = 0, n_heads = 0, n_kv_heads = 0, vocab_size = 0;
    int max_seq_len = 0;
    float rope_theta = 0;
    int rotary_dim = 0;
    float norm_eps = 1e-5f;
    ActivationType act = ActivationType::GELU;
    float qkv_clip = 0;
    bool tie_word_embeddings = false;

    static Config from_xalm(const XalmFile& xalm, int context = 0);
    xh_config to_abi() const;
};

struct InferenceState {
    explicit InferenceState(const Config& config) : _logits(config.vocab_size, 0.f) {}
    float* logits() { return _logits.data(); }
    const float* logits() const { return _logits.data(); }

private:
    std::vector<float> _logits;
};

class Model {
public:
    static Model from_xalm(const XalmFile& xalm, int context = 0, Device device = Device::HIP, int ordinal = 0);
    Model(Model&& o) noexcept;
    Model& operator=(Model&&) = delete;
    Model(const Model&) = delete;
    Model& operator=(const Model&) = delete;
    ~Model();

    Config config;

    void forward(InferenceState& s, int token, int pos, InferenceMode mode = InferenceMode::OUTPUT_LOGITS) const;
    // the prompt loop (src/main.cpp:94-100) in one call: HYDRATE tokens[0..n-1), the last with
    // logits into s (xh_prefill: batched passes of up to 64 tokens)
    void prefill(InferenceState& s, const std::vector<int>& tokens, int pos0) const;
    // greedy decode on the device (no host round trip per token); returns the tokens
    std::vector<int> decode_greedy(int pos, int n_steps, int stop_a = -1, int stop_b = -1) const;
    void fetch_logits(InferenceState& s) const;
    // run_perplexity's loop on the device (xh_perplexity): element i = Sampler::sample_prob of
    // tokens[i + 1] after forwarding tokens[i] at pos0 + i
    std::vector<float> token_probs(const std::vector<int>& tokens, int pos0) const;
    [[nodiscard]] size_t active_bytes(size_t pos) const;
    xh_ctx* ctx() const { return _ctx; }

private:
    Model(const Config& c, xh_ctx* ctx) : config(c), _ctx(ctx) {}
    xh_ctx* _ctx = nullptr;
};

// ---- tokenizer / sampler ------------------------------------------------------------------
struct TokenTrie {
    std::unordered_map<char, std::unique_ptr<TokenTrie>> children;
    int token_id = -1;
};

struct Tokenizer {
    std::vector<std::string> vocab;
    TokenTrie vocab_trie;
    int bos_id = -1, eos_id = -1, eot_id = -1, byte_fallback_start = -1;
    std::string byte_pieces[256];

    explicit Tokenizer(const XalmFile& data);
    std::vector<int> encode(const std::string& text, bool encode_bos) const;
    std::string decode_one(int prev_token, int token) const;
};

struct Sampler {
    explicit Sampler(const Config& c) : vocab_size(c.vocab_size) {}
    int vocab_size;
    int sample_argmax(const InferenceState& s) const;
    float sample_prob(int index, const InferenceState& s) const;
};

}  // namespace xalm
