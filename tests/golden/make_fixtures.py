"""Generate the committed golden fixtures under tests/golden/ (run in the dev container only).

What this produces, and why each piece pins parity:

* ``*.xalm`` model files written by the REFERENCE converter itself
  (``/root/reference/convert.py``: ``load_tokens`` :338-366, ``load_weights`` :696-852,
  ``save_xalm_binary`` :248-321) from small synthetic HF checkpoints (bf16 safetensors,
  seeded).  The converter source is read from /root/reference at run time and executed
  in memory; the only edit is swapping the quote style of four PEP-701 f-strings
  (convert.py:267,269,271,813) so that Python 3.10 can parse it.  Nothing of the
  reference is copied into this repository: only the converter's OUTPUT files are kept.
* ``hf_logits_*.npz``: per-position logits of HuggingFace ``MistralForCausalLM`` /
  ``LlamaForCausalLM`` (an independent implementation of the same math) built from the
  same config + safetensors.  They pin the CPU oracle (oracle/xalm_oracle.c), which
  restates ``src/infer.cpp``; the expected gap is the reference's fp16 KV-cache rounding
  (SURVEY §8c measured 4.8e-4 max-abs on a comparable fixture).
* ``tokenizer_golden.json``: prompt -> ids from a pure-Python restatement of the
  reference greedy-trie tokenizer (src/tokenizer.cpp:82-119), used to pin the C++ host
  tokenizer.

Run:  python tests/golden/make_fixtures.py      (needs /root/reference, torch, transformers)
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

# ---------------------------------------------------------------------------------------
# synthetic checkpoints
# ---------------------------------------------------------------------------------------
MODELS = {
    # Mistral-shaped: GQA 2 q-heads per kv head, head_dim 16, untied lm_head.
    "tiny_mistral": dict(arch="MistralForCausalLM", hidden_size=64, intermediate_size=192,
                         num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                         head_dim=16, vocab_size=300, max_position_embeddings=64,
                         rope_theta=1000000.0, rms_norm_eps=1e-5, hidden_act="silu",
                         tie_word_embeddings=False, seed=1234,
                         types=["f16", "bf16", "f32", "f8_e4m3", "f8_e5m2"]),
    # Llama-3-shaped head layout: 4 q-heads per kv head, head_dim 128 (as the real models),
    # tied embeddings (exercises `wcls = embed.weight`, src/model.cpp:428-430).
    "small_llama": dict(arch="LlamaForCausalLM", hidden_size=512, intermediate_size=512,
                        num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=1,
                        head_dim=128, vocab_size=320, max_position_embeddings=128,
                        rope_theta=500000.0, rms_norm_eps=1e-5, hidden_act="silu",
                        tie_word_embeddings=True, seed=4321, types=["f16"]),
}

PROMPT = "Q: What is the meaning of life? A: the answer is in the stars, or so they say."
# fixed token sequence used for the HF logits goldens (BOS + LCG ids, SURVEY §8d style)
def lcg_tokens(n, vocab, seed=7):
    out, s = [1], seed
    for _ in range(n - 1):
        s = (1103515245 * s + 12345) & 0x7FFFFFFF
        out.append(3 + s % (vocab - 3))
    return out


WORDS = ("the of and to in is was that for on as with by he at from his it an were are which this "
         "be or has had not but what all when there can who been one if will more so no out up "
         "about into than them some could time these two may then do first any my now such like "
         "our over man me even most made after also did many before must through back years where "
         "much your way well down should because each just those people how too little state good "
         "very make world still own see men work long get here between both life being under never "
         "day same another know while last might us great old year off come since against go came "
         "right used take three meaning answer stars say they Q A").split()


def make_vocab(vocab_size):
    """A sentencepiece-style byte-fallback vocab: <unk>,<s>,</s>, <0x00>..<0xFF>, then pieces."""
    toks = ["<unk>", "<s>", "</s>"] + [f"<0x{b:02X}>" for b in range(256)]
    pieces = []
    for w in WORDS:
        for p in ("▁" + w, w):
            if p not in pieces:
                pieces.append(p)
        for k in range(2, len(w)):
            if w[:k] not in pieces:
                pieces.append(w[:k])
    for c in "abcdefghijklmnopqrstuvwxyz?:.,":
        if c not in pieces:
            pieces.insert(0, c)
    pieces = ["▁"] + pieces
    need = vocab_size - len(toks)
    toks += pieces[:need]
    assert len(toks) == vocab_size, (len(toks), vocab_size)
    return toks


def write_checkpoint(d, spec):
    import torch
    from safetensors.torch import save_file

    g = torch.Generator().manual_seed(spec["seed"])
    H, I, L = spec["hidden_size"], spec["intermediate_size"], spec["num_hidden_layers"]
    nh, nkv, hd, V = spec["num_attention_heads"], spec["num_key_value_heads"], spec["head_dim"], spec["vocab_size"]

    def randn(*shape, std=0.02, mean=0.0):
        return (torch.randn(*shape, generator=g) * std + mean).to(torch.bfloat16)

    w = {"model.embed_tokens.weight": randn(V, H, std=1.0)}
    for l in range(L):
        p = f"model.layers.{l}."
        w[p + "input_layernorm.weight"] = randn(H, std=0.1, mean=1.0)
        w[p + "post_attention_layernorm.weight"] = randn(H, std=0.1, mean=1.0)
        w[p + "self_attn.q_proj.weight"] = randn(nh * hd, H, std=0.15)
        w[p + "self_attn.k_proj.weight"] = randn(nkv * hd, H, std=0.15)
        w[p + "self_attn.v_proj.weight"] = randn(nkv * hd, H, std=0.15)
        w[p + "self_attn.o_proj.weight"] = randn(H, nh * hd, std=0.08)
        w[p + "mlp.gate_proj.weight"] = randn(I, H, std=0.08)
        w[p + "mlp.up_proj.weight"] = randn(I, H, std=0.08)
        w[p + "mlp.down_proj.weight"] = randn(H, I, std=0.08)
    w["model.norm.weight"] = randn(H, std=0.1, mean=1.0)
    if not spec["tie_word_embeddings"]:
        w["lm_head.weight"] = randn(V, H, std=0.05)
    save_file(w, os.path.join(d, "model.safetensors"))

    cfg = {
        "architectures": [spec["arch"]],
        "model_type": "mistral" if spec["arch"].startswith("Mistral") else "llama",
        "hidden_size": H, "intermediate_size": I, "num_hidden_layers": L,
        "num_attention_heads": nh, "num_key_value_heads": nkv, "head_dim": hd,
        "vocab_size": V, "max_position_embeddings": spec["max_position_embeddings"],
        "bos_token_id": 1, "eos_token_id": 2, "rope_theta": spec["rope_theta"],
        "rms_norm_eps": spec["rms_norm_eps"], "hidden_act": spec["hidden_act"],
        "tie_word_embeddings": spec["tie_word_embeddings"], "torch_dtype": "bfloat16",
        "sliding_window": None,
    }
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(cfg, f, indent=1)

    toks = make_vocab(V)
    vocab = {t: i for i, t in enumerate(toks) if i >= 3}
    tok = {"model": {"type": "BPE", "byte_fallback": True, "vocab": vocab, "merges": []},
           "added_tokens": [{"id": i, "content": toks[i], "special": True} for i in range(3)]}
    with open(os.path.join(d, "tokenizer.json"), "w") as f:
        json.dump(tok, f, ensure_ascii=False)
    return cfg, w


# ---------------------------------------------------------------------------------------
# the reference converter, executed from /root/reference
# ---------------------------------------------------------------------------------------
def load_reference_converter():
    src_path = os.path.join(REF, "convert.py")
    with open(src_path) as f:
        src = f.read()
    # Python 3.10 cannot parse PEP-701 nested quotes; swap the inner quotes in memory.
    for a, b in (('["hash"]', "['hash']"), ('["offset"]', "['offset']"), ('["size"]', "['size']"),
                 ('.replace("torch.", "")', ".replace('torch.', '')")):
        assert a in src, a
        src = src.replace(a, b)
    sys.path.insert(0, REF)  # for `from quants import ...`
    mod = types.ModuleType("xalm_reference_convert")
    mod.__file__ = src_path
    exec(compile(src, src_path, "exec"), mod.__dict__)
    return mod


def convert(conv, ckpt_dir, out_path, xtype):
    """Mirror of convert.py's __main__ flow (:1131-1164) for one target type."""
    import torch
    config_file, tokenizer_file, model_files = conv.process_input(ckpt_dir)
    with open(config_file) as f:
        config = json.load(f)
    metadata = conv.Metadata(config)
    conv.args = argparse.Namespace(analyze=False)
    conv.config = config
    tokens = conv.load_tokens(tokenizer_file, metadata.vocab_size)
    tensors = conv.load_weights(model_files, conv.XType.parse(xtype), metadata,
                                config.get("tie_word_embeddings", None))
    tensors["tokenizer.tokens"] = torch.cat([torch.tensor([x for x in b] + [0], dtype=torch.uint8)
                                             for b in tokens])
    metadata.tensors["tokenizer.tokens"] = {"type": conv.XType.u8.name(),
                                            "shape": tensors["tokenizer.tokens"].shape}
    conv.save_xalm_binary(out_path, tensors, metadata)


# ---------------------------------------------------------------------------------------
# HF logits (independent implementation of the same forward)
# ---------------------------------------------------------------------------------------
def _register_f16kv():
    """HF eager attention with K/V rounded to fp16 after rope: the reference stores its KV
    cache as float16_t (src/infer.cpp:410-414), HF keeps fp32.  With this the remaining
    HF-vs-oracle gap is summation order only."""
    import torch
    from transformers import AttentionInterface

    def f16kv(module, query, key, value, attention_mask, scaling, dropout=0.0, **kw):
        # query [b, h, s, d]; key/value [b, kvh, s, d]; explicit causal softmax attention
        key = key.to(torch.float16).to(torch.float32)
        value = value.to(torch.float16).to(torch.float32)
        rep = query.shape[1] // key.shape[1]
        key = key.repeat_interleave(rep, dim=1)
        value = value.repeat_interleave(rep, dim=1)
        s = query.shape[2]
        scores = torch.matmul(query, key.transpose(2, 3)) * scaling
        causal = torch.triu(torch.ones(s, s, dtype=torch.bool), diagonal=1)
        scores = scores.masked_fill(causal, float("-inf"))
        p = torch.softmax(scores.float(), dim=-1)
        out = torch.matmul(p, value).transpose(1, 2).contiguous()
        return out, p

    AttentionInterface.register("f16kv", f16kv)


def hf_logits(cfg, weights, token_ids, attn="eager"):
    import torch
    import transformers
    kw = dict(hidden_size=cfg["hidden_size"], intermediate_size=cfg["intermediate_size"],
              num_hidden_layers=cfg["num_hidden_layers"], num_attention_heads=cfg["num_attention_heads"],
              num_key_value_heads=cfg["num_key_value_heads"], head_dim=cfg["head_dim"],
              vocab_size=cfg["vocab_size"], max_position_embeddings=cfg["max_position_embeddings"],
              rms_norm_eps=cfg["rms_norm_eps"], hidden_act=cfg["hidden_act"],
              tie_word_embeddings=cfg["tie_word_embeddings"],
              rope_parameters={"rope_type": "default", "rope_theta": cfg["rope_theta"]},
              attn_implementation=attn)
    if cfg["architectures"][0].startswith("Mistral"):
        model = transformers.MistralForCausalLM(transformers.MistralConfig(sliding_window=None, **kw))
    else:
        model = transformers.LlamaForCausalLM(transformers.LlamaConfig(**kw))
    sd = {k: v.to(torch.float32) for k, v in weights.items()}
    if cfg["tie_word_embeddings"]:
        sd["lm_head.weight"] = sd["model.embed_tokens.weight"]
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("rotary" in m or m == "lm_head.weight" for m in missing), missing
    model = model.to(torch.float32).eval()
    theta = model.config.rope_parameters["rope_theta"] if hasattr(model.config, "rope_parameters") else None
    assert theta is None or abs(theta - cfg["rope_theta"]) < 1e-3, theta
    with torch.no_grad():
        out = model(torch.tensor([token_ids]), use_cache=False).logits[0].float().numpy()
    return out


# ---------------------------------------------------------------------------------------
# tokenizer golden: restatement of src/tokenizer.cpp:82-119 (greedy longest trie match)
# ---------------------------------------------------------------------------------------
def ref_encode(vocab_bytes, text_bytes, bos_id, encode_bos=True):
    trie = {}
    for i, w in enumerate(vocab_bytes):           # tokenizer.cpp:86-96 (later ids overwrite)
        p = trie
        for c in w:
            p = p.setdefault(c, {})
        p[None] = i
    byte_fallback_start = vocab_bytes.index(b"<0x00>") if b"<0x00>" in vocab_bytes else -1
    out = [bos_id] if encode_bos else []
    i = 0
    while i < len(text_bytes):
        p, l, valid_l, valid = trie, 0, 0, None
        while i + l < len(text_bytes) and text_bytes[i + l] in p:
            p = p[text_bytes[i + l]]
            l += 1
            if None in p:
                valid, valid_l = p[None], l
        if valid is None:
            if byte_fallback_start >= 0:
                out.append(text_bytes[i] + byte_fallback_start)
            i += 1
        else:
            out.append(valid)
            i += valid_l
    return out


def read_xalm_tokens(path):
    """tokenizer.tokens (NUL-separated u8 tensor) of a .xalm file (layout: convert.py:248-321)."""
    with open(path, "rb") as f:
        blob = f.read()
    hsize = int.from_bytes(blob[:8], "little")
    header = json.loads(blob[8:hsize].split(b"\0", 1)[0])
    arch = [k for k in header if k != "xalm"][0]
    ti = header[arch]["tensors"]["tokenizer.tokens"]
    raw = blob[hsize + ti["offset"]: hsize + ti["offset"] + ti["size"]]
    return raw.split(b"\0")[:-1]


def main():
    import torch  # noqa: F401
    _register_f16kv()
    conv = load_reference_converter()
    tok_golden = {}
    for name, spec in MODELS.items():
        tmp = tempfile.mkdtemp(prefix=f"xalm_fix_{name}_")
        try:
            cfg, weights = write_checkpoint(tmp, spec)
            for t in spec["types"]:
                out = os.path.join(HERE, f"{name}_{t}.xalm")
                convert(conv, tmp, out, t)
                print("wrote", out, os.path.getsize(out))
            ids = lcg_tokens(24, spec["vocab_size"])
            logits = hf_logits(cfg, weights, ids)
            logits16 = hf_logits(cfg, weights, ids, attn="f16kv")
            np.savez_compressed(os.path.join(HERE, f"hf_logits_{name}.npz"),
                                tokens=np.array(ids, dtype=np.int32), logits=logits.astype(np.float32),
                                logits_f16kv=logits16.astype(np.float32))
            # tokenizer ids from the restated greedy trie over the vocab bytes the converter wrote
            vocab_b = read_xalm_tokens(os.path.join(HERE, f"{name}_{spec['types'][0]}.xalm"))
            for prompt in (PROMPT, "hello world", "Zebra! été"):
                tok_golden.setdefault(name, []).append(
                    {"prompt": prompt, "ids": ref_encode(vocab_b, prompt.encode("utf-8"), 1)})
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
    with open(os.path.join(HERE, "tokenizer_golden.json"), "w") as f:
        json.dump(tok_golden, f, indent=1, ensure_ascii=False)
    print("done")


if __name__ == "__main__":
    main()
