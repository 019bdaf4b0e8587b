// xalm_file.cpp — .xalm reader (Xalm::load, jubruckne/Xalm src/xalm.h:90-192) and Config.
#include <algorithm>
#include <cctype>
#include <cfloat>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>

#include "json.h"
#include "xalm.h"

namespace xalm {

// Type::parse, src/types.h:468-499 (case-insensitive names)
int parse_type(const std::string& s) {
    std::string u(s);
    std::transform(u.begin(), u.end(), u.begin(), [](unsigned char c) { return (char)std::toupper(c); });
    if (u == "F32") return XH_F32;
    if (u == "F16") return XH_F16;
    if (u == "BF16") return XH_BF16;
    if (u == "F8_E4M3") return XH_F8_E4M3;
    if (u == "F8_E5M2") return XH_F8_E5M2;
    if (u == "U8") return XH_U8;
    if (u == "Q8") return XH_Q8;
    // the converter's gguf blocks (convert.py:176-187); the reference runtime has no parser
    if (u == "Q8_0") return XH_Q8_0;
    if (u == "Q4_0") return XH_Q4_0;
    throw std::invalid_argument("invalid type: " + u);
}

size_t type_size(int type) {
    switch (type) {
        case XH_F32: return 4;
        case XH_F16: case XH_BF16: return 2;
        case XH_F8_E4M3: case XH_F8_E5M2: case XH_U8: case XH_Q8: return 1;
        default: return 0;
    }
}

XalmFile XalmFile::load(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw std::invalid_argument("cannot open " + path);
    const uint64_t file_size = (uint64_t)f.tellg();
    f.seekg(0);
    uint64_t header_size = 0;
    f.read((char*)&header_size, 8);
    if (!f || header_size == 0 || header_size > file_size - 8)
        throw std::invalid_argument("bad json size: " + std::to_string(header_size) + " for file size: " +
                                    std::to_string(file_size));
    std::string buf(header_size - 8, '\0');
    f.read(&buf[0], (std::streamsize)buf.size());
    buf.resize(strnlen(buf.data(), buf.size()));  // JSON ends at the first NUL of the padding
    const Json header = Json::parse(buf);
    const Json* xv = header.find("xalm");
    if (!xv) throw std::invalid_argument("invalid file format!");
    const Json* ver = xv->find("version");
    if (!ver || ver->as_int() != 1) throw std::invalid_argument("xalm version mismatch");

    XalmFile out;
    out.file_name = path;
    for (auto& kv : header.obj) {
        if (kv.first == "xalm") continue;
        if (kv.first != "LlamaForCausalLM" && kv.first != "MistralForCausalLM")
            throw std::invalid_argument("unsupported model architecture: " + kv.first);
        out.arch = kv.first;
        for (auto& m : kv.second.at("config").obj) out.metadata[m.first] = m.second.as_string();
        for (auto& t : kv.second.at("tensors").obj) {
            TensorInfo ti;
            ti.name = t.first;
            ti.type = parse_type(t.second.at("type").as_string());
            const Json& shape = t.second.at("shape");
            if (shape.arr.size() > 4) throw std::invalid_argument("shape exceeds 4 dimensions");
            for (auto& d : shape.arr) ti.shape.push_back((int)d.as_int());
            const long long off = t.second.contains("offset") ? t.second.at("offset").as_int() : -1;
            const long long size = t.second.contains("size") ? t.second.at("size").as_int() : -1;
            if (off < 0) throw std::invalid_argument("bad offset");
            if (size < 0) throw std::invalid_argument("bad size");
            if ((uint64_t)(off + size) + header_size > file_size)
                throw std::invalid_argument("offset out of range for " + ti.name);
            ti.offset = (size_t)(header_size + off);
            ti.size = (size_t)size;
            out.tensors[ti.name] = ti;
        }
    }
    if (out.arch.empty()) throw std::invalid_argument("no model in file");
    return out;
}

void XalmFile::read(const TensorInfo& ti, void* dst) const {
    std::ifstream f(file_name, std::ios::binary);
    f.seekg((std::streamoff)ti.offset);
    f.read((char*)dst, (std::streamsize)ti.size);
    if (!f) throw std::runtime_error("short read of " + ti.name);
}

std::vector<uint8_t> XalmFile::read(const std::string& name) const {
    const TensorInfo& ti = tensors.at(name);
    std::vector<uint8_t> buf(ti.size);
    read(ti, buf.data());
    return buf;
}

const std::string& XalmFile::meta(const std::string& key) const {
    auto it = metadata.find(key);
    if (it == metadata.end()) throw std::out_of_range("missing metadata key " + key);
    return it->second;
}

std::string XalmFile::meta_or(const std::string& key, const std::string& dflt) const {
    auto it = metadata.find(key);
    return it == metadata.end() ? dflt : it->second;
}

// Config::from_xalm, src/model.h:44-90
Config Config::from_xalm(const XalmFile& x, const int context) {
    Config c;
    c.dim = std::stoi(x.meta("dim"));
    c.hidden_dim = std::stoi(x.meta("hidden_dim"));
    c.head_dim = std::stoi(x.meta("head_dim"));
    c.n_layers = std::stoi(x.meta("n_layers"));
    c.n_heads = std::stoi(x.meta("n_heads"));
    c.n_kv_heads = std::stoi(x.meta("n_kv_heads"));
    c.vocab_size = std::stoi(x.meta("vocab_size"));
    c.max_seq_len = std::min(std::stoi(x.meta("max_seq_len")), 4096);
    if (context) c.max_seq_len = context;
    c.rope_theta = std::stof(x.meta("rope_theta"));
    c.rotary_dim = std::stoi(x.meta("rotary_dim"));
    c.norm_eps = std::stof(x.meta_or("norm_eps", "1e-5"));
    const std::string act = x.meta_or("act_type", "gelu");
    if (act == "silu") c.act = ActivationType::SILU;
    else {
        if (act != "gelu") fprintf(stderr, "unsupported act_type, defaulting to gelu\n");
        c.act = ActivationType::GELU;
    }
    const std::string norm = x.meta_or("norm_type", "rmsnorm");
    if (norm != "rmsnorm") fprintf(stderr, "unsupported norm_type, defaulting to rmsnorm\n");
    c.qkv_clip = x.metadata.count("qkv_clip") ? std::stof(x.meta("qkv_clip")) : FLT_MAX;
    c.tie_word_embeddings = x.meta("tie_word_embeddings") == "True";
    return c;
}

xh_config Config::to_abi() const {
    xh_config c{};
    c.dim = dim; c.hidden_dim = hidden_dim; c.head_dim = head_dim; c.n_layers = n_layers;
    c.n_heads = n_heads; c.n_kv_heads = n_kv_heads; c.vocab_size = vocab_size; c.max_seq_len = max_seq_len;
    c.rope_theta = rope_theta; c.rotary_dim = rotary_dim; c.norm_eps = norm_eps; c.act = (int)act;
    c.qkv_clip = qkv_clip; c.tie_word_embeddings = tie_word_embeddings ? 1 : 0;
    return c;
}

}  // namespace xalm
