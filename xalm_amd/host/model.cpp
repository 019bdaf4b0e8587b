// model.cpp — Model::from_xalm / forward over the C ABI (jubruckne/Xalm src/model.cpp:48-122),
// Tokenizer (src/tokenizer.cpp) and Sampler (src/sampler.cpp).
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <limits>
#include <stdexcept>

#include "xalm.h"

namespace xalm {

namespace {
void check(int rc, xh_ctx* ctx, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + xh_last_error(ctx));
}
}  // namespace

// Model::from_xalm, src/model.cpp:48-118: the same tensor names and shape checks; the weights
// stream from the file into device memory through xh_upload_file (mapped, pinned and DMAd; no host
// Tensor buffers).
Model Model::from_xalm(const XalmFile& xalm, const int context, const Device device, const int ordinal) {
    if (device != Device::HIP)
        throw std::invalid_argument(
            "-d cpu: the reference CPU forward is not part of this build (its restatement is the test oracle, "
            "oracle/); use -d hip");
    const Config c = Config::from_xalm(xalm, context);
    xh_config abi = c.to_abi();
    xh_ctx* ctx = nullptr;
    check(xh_create(&abi, ordinal, &ctx), nullptr, "xh_create");
    Model m(c, ctx);
    auto load = [&](const std::string& name, int kind, int layer, std::vector<int> shape) {
        const TensorInfo& ti = xalm.tensors.at(name);
        // gguf blocks (convert.py:176-187): the header holds the byte shape, 32 elements per block
        if ((ti.type == XH_Q8_0 || ti.type == XH_Q4_0) && shape.size() == 2 && shape[1] % 32 == 0)
            shape[1] = shape[1] / 32 * (ti.type == XH_Q8_0 ? 34 : 18);
        if (ti.shape != shape) {
            std::string a, b;
            for (int v : ti.shape) a += std::to_string(v) + ",";
            for (int v : shape) b += std::to_string(v) + ",";
            throw std::invalid_argument("shape mismatch for " + name + ": [" + a + "] vs [" + b + "] expected!");
        }
        check(xh_upload_file(ctx, kind, layer, ti.type, xalm.file_name.c_str(), ti.offset, ti.size), ctx,
              name.c_str());
    };
    const int q_dim = c.n_heads * c.head_dim, kv_dim = c.n_kv_heads * c.head_dim;
    load("embed.weight", XH_EMBED, 0, {c.vocab_size, c.dim});
    for (int i = 0; i < c.n_layers; ++i) {
        const std::string p = "l." + std::to_string(i) + ".";
        load(p + "attn.norm.weight", XH_ATTN_NORM, i, {c.dim});
        load(p + "mlp.norm.weight", XH_FFN_NORM, i, {c.dim});
        load(p + "attn.q.weight", XH_WQ, i, {q_dim, c.dim});
        load(p + "attn.k.weight", XH_WK, i, {kv_dim, c.dim});
        load(p + "attn.v.weight", XH_WV, i, {kv_dim, c.dim});
        load(p + "attn.down.weight", XH_WO, i, {c.dim, q_dim});
        load(p + "mlp.gate.weight", XH_W1, i, {c.hidden_dim, c.dim});
        load(p + "mlp.down.weight", XH_W2, i, {c.dim, c.hidden_dim});
        load(p + "mlp.up.weight", XH_W3, i, {c.hidden_dim, c.dim});
    }
    load("output.norm.weight", XH_FINAL_NORM, 0, {c.dim});
    if (!c.tie_word_embeddings) load("output.weight", XH_WCLS, 0, {c.vocab_size, c.dim});
    return m;
}

Model::Model(Model&& o) noexcept : config(o.config), _ctx(o._ctx) { o._ctx = nullptr; }

Model::~Model() {
    if (_ctx) xh_destroy(_ctx);
}

void Model::forward(InferenceState& s, const int token, const int pos, const InferenceMode mode) const {
    float* out = mode == InferenceMode::OUTPUT_LOGITS ? s.logits() : nullptr;
    check(xh_forward(_ctx, token, pos, (int)mode, out), _ctx, "xh_forward");
}

void Model::prefill(InferenceState& s, const std::vector<int>& tokens, const int pos0) const {
    if (tokens.empty()) return;
    check(xh_prefill(_ctx, tokens.data(), (int)tokens.size(), pos0, 1, s.logits()), _ctx, "xh_prefill");
}

std::vector<int> Model::decode_greedy(const int pos, const int n_steps, const int stop_a, const int stop_b) const {
    std::vector<int> toks((size_t)std::max(n_steps, 1));
    int done = 0;
    check(xh_decode_greedy(_ctx, pos, n_steps, stop_a, stop_b, toks.data(), &done), _ctx, "xh_decode_greedy");
    toks.resize((size_t)done);
    return toks;
}

std::vector<float> Model::token_probs(const std::vector<int>& tokens, const int pos0) const {
    if (tokens.size() < 2) return {};
    std::vector<float> p(tokens.size() - 1);
    check(xh_perplexity(_ctx, tokens.data(), (int)tokens.size(), pos0, p.data()), _ctx, "xh_perplexity");
    return p;
}

void Model::fetch_logits(InferenceState& s) const { check(xh_get_logits(_ctx, s.logits()), _ctx, "xh_get_logits"); }

size_t Model::active_bytes(const size_t pos) const { return xh_active_bytes(_ctx, pos); }

// ---- Tokenizer, src/tokenizer.cpp:23-119 ---------------------------------------------------
namespace {
std::vector<int> parse_ids(const std::string& input) {
    std::vector<int> r;
    if (!input.empty() && input.front() == '[' && input.back() == ']') {
        std::string t = input.substr(1, input.size() - 2);
        size_t i = 0;
        while (i < t.size()) {
            size_t j = t.find(',', i);
            if (j == std::string::npos) j = t.size();
            r.push_back(std::stoi(t.substr(i, j - i)));
            i = j + 1;
        }
    } else {
        r.push_back(std::stoi(input));
    }
    return r;
}
}  // namespace

Tokenizer::Tokenizer(const XalmFile& data) {
    bos_id = parse_ids(data.meta("bos_token_id"))[0];
    eos_id = parse_ids(data.meta("eos_token_id"))[0];
    const TensorInfo& ti = data.tensors.at("tokenizer.tokens");
    if (ti.type != XH_U8) throw std::invalid_argument("tokenizer.tokens must be U8");
    const std::vector<uint8_t> raw = data.read("tokenizer.tokens");
    const char* p = (const char*)raw.data();
    const char* end = p + raw.size();
    while (p < end) {
        const char* s = p;
        while (p < end && *p != '\0') p++;
        vocab.emplace_back(s, (size_t)(p - s));
        p++;
    }
    for (size_t i = 0; i < vocab.size(); i++) {
        if (vocab[i] == "<0x00>") byte_fallback_start = (int)i;
        else if (vocab[i] == "<|eot_id|>" || vocab[i] == "<|end|>" || vocab[i] == "<|im_end|>") eot_id = (int)i;
    }
    for (int i = 0; i < 256; i++) byte_pieces[i] = std::string(1, (char)i);
    for (size_t i = 0; i < vocab.size(); i++) {
        TokenTrie* n = &vocab_trie;
        for (char ch : vocab[i]) {
            auto& child = n->children[ch];
            if (!child) child = std::make_unique<TokenTrie>();
            n = child.get();
        }
        n->token_id = (int)i;
    }
}

std::string Tokenizer::decode_one(const int prev_token, const int token) const {
    const std::string& piece = vocab[token];
    if (prev_token == bos_id && !piece.empty() && piece[0] == ' ') return piece.substr(1);
    if (byte_fallback_start >= 0 && token >= byte_fallback_start && token - byte_fallback_start < 256)
        return byte_pieces[token - byte_fallback_start];
    return piece;
}

// greedy longest match over the vocab trie with byte fallback (src/tokenizer.cpp:82-119)
std::vector<int> Tokenizer::encode(const std::string& text, const bool encode_bos) const {
    std::vector<int> out;
    if (encode_bos) out.push_back(bos_id);
    for (size_t i = 0; i < text.size();) {
        size_t l = 0, valid_l = 0;
        const TokenTrie* p = &vocab_trie;
        const TokenTrie* valid_p = nullptr;
        while (i + l < text.size()) {
            auto it = p->children.find(text[i + l]);
            if (it == p->children.end()) break;
            p = it->second.get();
            l += 1;
            if (p->token_id >= 0) { valid_p = p; valid_l = l; }
        }
        if (!valid_p) {
            if (byte_fallback_start >= 0) out.push_back((unsigned char)text[i] + byte_fallback_start);
            i += 1;
        } else {
            out.push_back(valid_p->token_id);
            i += valid_l;
        }
    }
    return out;
}

// ---- Sampler, src/sampler.cpp:3-30 (max starts at FLT_MIN; first maximum wins) -------------
int Sampler::sample_argmax(const InferenceState& s) const {
    const float* logits = s.logits();
    int argmax = 0;
    float max_val = std::numeric_limits<float>::min();
    for (int i = 0; i < vocab_size; ++i)
        if (logits[i] > max_val) { max_val = logits[i]; argmax = i; }
    return argmax;
}

float Sampler::sample_prob(const int index, const InferenceState& s) const {
    const float* logits = s.logits();
    float max_val = std::numeric_limits<float>::min();
    for (int i = 0; i < vocab_size; ++i)
        if (logits[i] > max_val) max_val = logits[i];
    float sum = 0;
    for (int i = 0; i < vocab_size; ++i) sum += expf(logits[i] - max_val);
    return expf(logits[index] - max_val) / sum;
}

}  // namespace xalm
