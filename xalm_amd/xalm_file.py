"""Python reader for the .xalm container (host-side support for tests and bench).

Mirrors `Xalm::load` (jubruckne/Xalm src/xalm.h:90-192) and `Config::from_xalm`
(src/model.h:44-90).  Layout written by convert.py `save_xalm_binary` (:248-321):
  u64 header_size (total bytes before the data blob, 4096-aligned)
  JSON {"xalm": {"version": 1}, "<Arch>": {"config": {...strings...},
                                            "tensors": {name: {type, shape, offset, size, hash}}}}
  zero padding up to header_size, then tensor data at header_size + offset (32-B aligned).
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass

import numpy as np

from . import _lib as L

SUPPORTED_ARCHS = ("LlamaForCausalLM", "MistralForCausalLM")  # src/xalm.h:141


@dataclass
class TensorInfo:
    name: str
    type: str
    shape: tuple
    offset: int  # absolute file offset
    size: int


class XalmFile:
    def __init__(self, path: str):
        self.path = path
        with open(path, "rb") as f:
            head = f.read(8)
            if len(head) != 8:
                raise ValueError("file too short")
            (hsize,) = struct.unpack("<Q", head)
            f.seek(0, 2)
            fsize = f.tell()
            if hsize == 0 or hsize > fsize:
                raise ValueError(f"bad json size: {hsize} for file size: {fsize}")
            f.seek(8)
            raw = f.read(hsize - 8)
        header = json.loads(raw.split(b"\0", 1)[0].decode("utf-8"))
        if "xalm" not in header:
            raise ValueError("invalid file format!")
        if header["xalm"].get("version", 0) != 1:
            raise ValueError(f"xalm version mismatch: {header['xalm'].get('version')}")
        self.metadata = None
        self.arch = None
        self.tensors: dict[str, TensorInfo] = {}
        for arch, val in header.items():
            if arch == "xalm":
                continue
            if arch not in SUPPORTED_ARCHS:
                raise ValueError(f"unsupported model architecture: {arch}")
            self.arch = arch
            self.metadata = val["config"]
            for name, t in val["tensors"].items():
                shape = tuple(int(s) for s in t["shape"])
                if len(shape) > 4:
                    raise ValueError("shape exceeds 4 dimensions")
                off, size = int(t.get("offset", -1)), int(t.get("size", -1))
                if off < 0 or size < 0 or hsize + off + size > fsize:
                    raise ValueError(f"offset out of range for {name}")
                self.tensors[name] = TensorInfo(name, t["type"].upper(), shape, hsize + off, size)
        self._mm = np.memmap(path, dtype=np.uint8, mode="r")

    def raw(self, name: str) -> np.ndarray:
        ti = self.tensors[name]
        return self._mm[ti.offset: ti.offset + ti.size]

    def dtype(self, name: str) -> int:
        return L.DTYPE_BY_NAME[self.tensors[name].type]

    def config(self, context: int = 0) -> L.XhConfig:
        """Config::from_xalm (src/model.h:44-90): max_seq_len capped at 4096 unless `context`."""
        m = self.metadata
        c = L.XhConfig()
        c.dim = int(m["dim"])
        c.hidden_dim = int(m["hidden_dim"])
        c.head_dim = int(m["head_dim"])
        c.n_layers = int(m["n_layers"])
        c.n_heads = int(m["n_heads"])
        c.n_kv_heads = int(m["n_kv_heads"])
        c.vocab_size = int(m["vocab_size"])
        c.max_seq_len = min(int(m["max_seq_len"]), 4096)
        if context:
            c.max_seq_len = context
        c.rope_theta = float(m["rope_theta"])
        c.rotary_dim = int(m["rotary_dim"])
        c.norm_eps = float(m.get("norm_eps", "1e-5"))
        c.act = L.ACT_SILU if m.get("act_type", "gelu") == "silu" else L.ACT_GELU
        c.qkv_clip = float(m["qkv_clip"]) if "qkv_clip" in m else float(np.finfo(np.float32).max)
        c.tie_word_embeddings = 1 if m["tie_word_embeddings"] == "True" else 0
        return c

    def tokens(self) -> list[bytes]:
        """tokenizer.tokens: NUL-separated vocab (src/tokenizer.cpp:23-47)."""
        return bytes(self.raw("tokenizer.tokens")).split(b"\0")[:-1]

    def layer_tensors(self, layer: int) -> dict[int, str]:
        """Tensor names per kind, as Model::from_xalm loads them (src/model.cpp:83-114)."""
        p = f"l.{layer}."
        return {L.ATTN_NORM: p + "attn.norm.weight", L.FFN_NORM: p + "mlp.norm.weight",
                L.WQ: p + "attn.q.weight", L.WK: p + "attn.k.weight", L.WV: p + "attn.v.weight",
                L.WO: p + "attn.down.weight", L.W1: p + "mlp.gate.weight", L.W2: p + "mlp.down.weight",
                L.W3: p + "mlp.up.weight"}

    def global_tensors(self, tie: bool) -> dict[int, str]:
        return {L.EMBED: "embed.weight", L.FINAL_NORM: "output.norm.weight",
                L.WCLS: "embed.weight" if tie else "output.weight"}
