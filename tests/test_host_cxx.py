"""C++ host (libxalm_host.so, bin/xalm): reader, tokenizer, CLI.

CPU part: the C++ .xalm reader and Config::from_xalm agree with the Python reader; the
greedy-trie tokenizer reproduces tokenizer_golden.json (ids from a restatement of
src/tokenizer.cpp:82-119 over the converter-written vocab).
GPU part: `xalm` completion / perplexity on a fixture agree with the CPU oracle.
"""
import ctypes
import json
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, fixture_path
from xalm_amd import _lib as L
from xalm_amd.xalm_file import XalmFile

HOST_SO = os.path.join(ROOT, "xalm_amd", "lib", "libxalm_host.so")
CLI = os.path.join(ROOT, "xalm_amd", "bin", "xalm")


def host():
    lib = ctypes.CDLL(HOST_SO)
    lib.xalm_read_config.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(L.XhConfig)]
    lib.xalm_encode.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    lib.xalm_host_last_error.restype = ctypes.c_char_p
    return lib


@pytest.mark.parametrize("name", ["tiny_mistral_f16", "tiny_mistral_f8_e4m3", "small_llama_f16"])
@pytest.mark.parametrize("context", [0, 16])
def test_cxx_config_matches_python(name, context):
    path = fixture_path(name + ".xalm")
    c = L.XhConfig()
    assert host().xalm_read_config(path.encode(), context, ctypes.byref(c)) == 0
    p = XalmFile(path).config(context)
    for f, _ in L.XhConfig._fields_:
        assert getattr(c, f) == getattr(p, f), f


def test_cxx_tokenizer_matches_golden():
    gold = json.load(open(fixture_path("tokenizer_golden.json")))
    lib = host()
    for model, cases in gold.items():
        t = "f16"
        path = fixture_path(f"{model}_{t}.xalm").encode()
        for case in cases:
            out = (ctypes.c_int * 512)()
            n = ctypes.c_int(0)
            assert lib.xalm_encode(path, case["prompt"].encode("utf-8"), 1, out, 512, ctypes.byref(n)) == 0
            assert list(out[: n.value]) == case["ids"], case["prompt"]


def test_cxx_reader_rejects_garbage(tmp_path):
    p = tmp_path / "bad.xalm"
    p.write_bytes(b"\x10" + b"\x00" * 30)
    c = L.XhConfig()
    lib = host()
    assert lib.xalm_read_config(str(p).encode(), 0, ctypes.byref(c)) != 0
    assert lib.xalm_host_last_error()


def test_cli_rejects_cpu_device_and_bad_args():
    r = subprocess.run([CLI, fixture_path("tiny_mistral_f16.xalm"), "-d", "cpu", "-n", "2"], capture_output=True,
                       text=True)
    assert r.returncode != 0 and "oracle" in r.stderr
    r = subprocess.run([CLI, fixture_path("tiny_mistral_f16.xalm"), "-q", "1"], capture_output=True, text=True)
    assert r.returncode != 0 and "Usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("device_loop", ["0", "1"])
def test_cli_completion_matches_oracle(device_loop):
    from oracle import oracle as O
    path = fixture_path("tiny_mistral_f16.xalm")
    r = subprocess.run([CLI, path, "-n", "12", "-i", "the answer is", "-g", device_loop], capture_output=True,
                       timeout=120)
    out_txt = r.stdout.decode("utf-8", errors="replace")
    assert r.returncode == 0, r.stderr.decode(errors="replace")
    ids = [int(v) for v in re.search(r"tokens: \[([0-9,]*)\]", out_txt).group(1).split(",")]
    xf = XalmFile(path)
    om = O.OracleModel.from_xalm(xf)
    lib = host()
    out = (ctypes.c_int * 64)()
    n = ctypes.c_int(0)
    assert lib.xalm_encode(path.encode(), b"the answer is", 1, out, 64, ctypes.byref(n)) == 0
    prompt = list(out[: n.value])
    assert ids[: len(prompt)] == prompt
    for pos, tok in enumerate(ids[:-1]):
        om.forward(tok, pos)
        if pos >= len(prompt) - 1:
            lg = om.logits()
            top2 = np.sort(lg)[-2:]
            if top2[1] - top2[0] > 1e-3:
                assert ids[pos + 1] == O.sample_argmax(lg), pos


@pytest.mark.gpu
def test_cli_perplexity_matches_oracle():
    from oracle import oracle as O
    # tiny_mistral: logits of O(1), so no probability underflows to 0 in sample_prob (on the
    # small_llama fixture, |logits| ~ 87 and the reference's own perplexity is inf)
    path = fixture_path("tiny_mistral_f16.xalm")
    text = "Q: What is the meaning of life? A: the answer is in the stars"
    r = subprocess.run([CLI, path, "-m", "perplexity", "-i", text], capture_output=True, timeout=120)
    out_txt = r.stdout.decode("utf-8", errors="replace")
    assert r.returncode == 0, r.stderr.decode(errors="replace")
    m = re.search(r"^perplexity: (\S+)$", out_txt, re.M)
    assert m, out_txt
    ppl = float(m.group(1))
    lib = host()
    out = (ctypes.c_int * 128)()
    n = ctypes.c_int(0)
    assert lib.xalm_encode(path.encode(), text.encode(), 1, out, 128, ctypes.byref(n)) == 0
    ids = list(out[: n.value])
    om = O.OracleModel.from_xalm(XalmFile(path))
    s = 0.0
    for pos in range(len(ids) - 1):
        om.forward(ids[pos], pos)
        s += np.log(O.sample_prob(om.logits(), ids[pos + 1]))
    ref = float(np.exp(-s / (len(ids) - 1)))
    assert np.isfinite(ref) and abs(ppl - ref) <= 1e-3 * ref
