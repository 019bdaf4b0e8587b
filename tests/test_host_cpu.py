"""CPU-side tests: .xalm reader, config resolution, and the C ABI library surface.

No compute runs here (no GPU in the dev container): the library must load, export every
symbol include/*.h declares, and fail cleanly (an error code, no crash) without a device.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, fixture_path
from xalm_amd import _lib as L
from xalm_amd.xalm_file import XalmFile


def declared_functions(header):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(xh_\w+|xalm_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    names = declared_functions(os.path.join(ROOT, "include", "xalm_hip.h"))
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), n


def test_library_needs_no_vendor_gemm():
    """hipBLASLt (XH_OPT_PREFILL 4 only) is dlopen'ed on first use: it is not a link dependency
    of the product library (ELF DT_NEEDED entries read straight from the file)."""
    import struct
    data = open(L.HIP_LIB_PATH, "rb").read()
    assert data[:4] == b"\x7fELF" and data[4] == 2  # ELF64, little endian
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    dyn = [s for s in secs if s[1] == 6]  # SHT_DYNAMIC
    assert dyn
    _, _, _, _, off, size, link, _, _, entsize = dyn[0]
    stroff = secs[link][4]
    needed = []
    for i in range(size // entsize):
        tag, val = struct.unpack_from("<qQ", data, off + i * entsize)
        if tag == 1:  # DT_NEEDED
            needed.append(data[stroff + val:data.index(b"\0", stroff + val)].decode())
    assert any(n.startswith("libamdhip64") for n in needed), needed
    assert not any("blas" in n for n in needed), needed


def test_host_library_exports_declared_symbols():
    hdr = os.path.join(ROOT, "include", "xalm_host.h")
    so = os.path.join(ROOT, "xalm_amd", "lib", "libxalm_host.so")
    if not os.path.exists(hdr):
        pytest.skip("host header not present")
    lib = ctypes.CDLL(so)
    for n in declared_functions(hdr):
        assert hasattr(lib, n), n


def test_create_without_device_fails_cleanly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    cfg = xf.config()
    ctx = ctypes.c_void_p()
    rc = L.lib().xh_create(ctypes.byref(cfg), 0, ctypes.byref(ctx))
    assert rc != 0 and not ctx
    assert L.lib().xh_last_error(None)


def test_op_args_validated_before_device_use():
    x = np.zeros(17, np.float32)
    w = np.zeros(17 * 4, np.uint16)
    with pytest.raises(L.XhError):
        L.op_matmul(x, w, L.F16, 17, 4)  # n % 16 != 0
    with pytest.raises(L.XhError):
        L.op_matmul(np.zeros(16, np.float32), np.zeros(64, np.uint16), 5, 16, 4)  # bad dtype


@pytest.mark.parametrize("name", ["tiny_mistral_f16", "tiny_mistral_bf16", "tiny_mistral_f32",
                                  "tiny_mistral_f8_e4m3", "tiny_mistral_f8_e5m2", "small_llama_f16",
                                  "tiny_mistral_q8_0", "tiny_mistral_q4_0", "small_llama_q8_0"])
def test_xalm_reader(name):
    xf = XalmFile(fixture_path(name + ".xalm"))
    c = xf.config()
    assert xf.arch in ("MistralForCausalLM", "LlamaForCausalLM")
    assert len(xf.tokens()) == c.vocab_size
    for layer in range(c.n_layers):
        for kind, tn in xf.layer_tensors(layer).items():
            ti = xf.tensors[tn]
            dt = xf.dtype(tn)
            if dt in L.GQ_BLOCK_BYTES:
                # gguf blocks: the header shape is [rows, bytes per row] (quants.py byte shape)
                assert ti.size == int(np.prod(ti.shape)) and ti.shape[-1] % L.GQ_BLOCK_BYTES[dt] == 0
            else:
                assert ti.size == int(np.prod(ti.shape)) * L.DTYPE_SIZE[dt]
            assert ti.offset % 32 == 0  # convert.py align_offset
    # norms stay bf16 whatever the matrix type (convert.py:770-774)
    assert xf.tensors["l.0.attn.norm.weight"].type == "BF16"
    if "q8_0" in name or "q4_0" in name:  # no boost for gguf targets (convert.py:729-744)
        want = "Q8_0" if "q8_0" in name else "Q4_0"
        assert xf.tensors["embed.weight"].type == want and xf.tensors["l.0.mlp.down.weight"].type == want
    if "f8_e4m3" in name:  # embed/lm_head boosted to bf16 (convert.py:729-744)
        assert xf.tensors["embed.weight"].type == "BF16"
        assert xf.tensors["l.0.attn.q.weight"].type == "F8_E4M3"


def test_config_context_override_and_cap():
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    assert xf.config().max_seq_len == 64
    assert xf.config(context=16).max_seq_len == 16
    c = xf.config()
    assert c.act == L.ACT_SILU and abs(c.rope_theta - 1e6) < 1 and c.rotary_dim == 16
    assert c.tie_word_embeddings == 0
    assert XalmFile(fixture_path("small_llama_f16.xalm")).config().tie_word_embeddings == 1


def test_reader_rejects_garbage(tmp_path):
    p = tmp_path / "bad.xalm"
    p.write_bytes(b"\x00" * 16)
    with pytest.raises(ValueError):
        XalmFile(str(p))
