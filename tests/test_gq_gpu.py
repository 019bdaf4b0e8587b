"""gguf block formats (Q8_0 / Q4_0) on the device vs the CPU oracle.

The oracle decodes the converter's block bytes exactly as quants.py (tests/test_gq_cpu.py pins
that); the device repacks them into planar rows and scales each chunk's partial dot product
by its block's d.  Bars: matvec |gpu - cpu| <= 2e-6 * sum|w x| + 1e-7 (tests/test_ops_gpu.py);
whole forward logits within 1e-3 * max(1, max|logit|) (tests/test_forward_gpu.py).
"""
import numpy as np
import pytest

import bench
from bars import check, check_logp
from conftest import fixture_path
from oracle import oracle as O
from xalm_amd import _lib as L
from xalm_amd.model import InferenceState, Model
from xalm_amd.xalm_file import XalmFile

pytestmark = pytest.mark.gpu

GQ = [L.Q8_0, L.Q4_0]


def dequant(dtype, w):
    """|weights| scale for the tolerance: the block values d*q (quants.py dequantize_blocks)."""
    bs = L.GQ_BLOCK_BYTES[dtype]
    blk = np.ascontiguousarray(w).reshape(-1, bs)
    d = blk[:, :2].copy().view(np.float16).astype(np.float32)
    if dtype == L.Q8_0:
        q = blk[:, 2:].view(np.int8).astype(np.float32)
    else:
        q = np.concatenate([blk[:, 2:] & 15, blk[:, 2:] >> 4], axis=1).astype(np.float32) - 8
    return (d * q).reshape(w.shape[0], -1)


def tol(ref):  # the north-star bar (synthetic block models); fixtures: bars.check
    return 1e-3 * max(1.0, float(np.abs(ref).max()))


@pytest.mark.parametrize("dtype", GQ)
@pytest.mark.parametrize("n,d", [(64, 32), (512, 96), (4096, 64), (1536, 300), (14336, 8), (4096, 1025)])
def test_matmul_blocks(dtype, n, d):
    rng = np.random.default_rng(n + 13 * d + dtype)
    wf = (rng.standard_normal((d, n)) * 0.05).astype(np.float32)
    w = O.quantize_gq(dtype, wf)
    x = rng.standard_normal(n).astype(np.float32)
    got = L.op_matmul(x, w, dtype, n, d)
    cpu = O.matmul(x, w, dtype, n, d)
    mag = np.abs(dequant(dtype, w)).astype(np.float64) @ np.abs(x.astype(np.float64))
    assert np.all(np.abs(got - cpu) <= 2e-6 * mag + 1e-7), np.abs(got - cpu).max()


@pytest.mark.parametrize("name", ["tiny_mistral_q8_0", "tiny_mistral_q4_0", "small_llama_q8_0"])
@pytest.mark.parametrize("fuse", [1, 0])
def test_forward_on_converter_blocks(name, fuse):
    # every fixture position with logits vs the oracle, then the batched prompt path (f32-input
    # MFMA GEMMs decoding the blocks, prefill.h) and the device greedy loop
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf)
    gm.set_option(L.OPT_FUSE_ATTN_WO, fuse)
    om = O.OracleModel.from_xalm(xf)
    st = InferenceState(gm.config)
    toks = [1] + [3 + (i * 37) % (gm.config.vocab_size - 3) for i in range(20)]
    for pos, tok in enumerate(toks):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        check(st.logits(), om.logits(), name, "loop", pos)
    # prompt path and the device greedy loop
    gm.reset()
    om.reset()
    gm.prefill(toks[:9], 0, st)
    for pos, tok in enumerate(toks[:9]):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == 8 else L.HYDRATE_KV_CACHE)
    check(st.logits(), om.logits(), name, "prefill")
    out = gm.decode_greedy(9, 6)
    pos = 9
    for t in out:
        lg = om.logits()
        if np.sort(lg)[-1] - np.sort(lg)[-2] > 1e-3:
            assert t == O.sample_argmax(lg)
        om.forward(t, pos)
        pos += 1
    gm.close()
    om.close()


@pytest.mark.parametrize("dim,hidden,layers", [(2048, 4096, 2), (4096, 2048, 1)])
@pytest.mark.parametrize("dtype", GQ)
def test_synthetic_blocks_forward(dtype, dim, hidden, layers):
    # device-generated blocks (synth_gq_kernel) equal the oracle's (xo_fill_synthetic): the
    # logits agree; dims that take the long-row matvec shapes, and (dim 4096) the pipelined
    # block shapes for qkv, W1/W3 and lm_head (n = 4096) and Wo / W2 (n = 2048)
    w = dict(dim=dim, hidden=hidden, layers=layers, heads=16, kv_heads=4, head_dim=128, vocab=1000, msl=256,
             theta=1e6, wdt=dtype, edt=dtype, cdt=dtype)
    c = bench.make_config(w)
    gm, om = Model(c), O.OracleModel(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
        rows, cols = bench.tensor_shape(c, kind)
        om.set_tensor(kind, layer, dt, O.synthetic(rows, cols, dt, seed, mean, std))
    st = InferenceState(c)
    for pos, tok in enumerate([1, 17, 999, 3, 512]):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        ref = om.logits()
        assert np.abs(st.logits() - ref).max() <= tol(ref), pos
    gm.close()
    om.close()


def test_block_upload_checks():
    xf = XalmFile(fixture_path("tiny_mistral_q8_0.xalm"))
    gm = Model.from_xalm(xf)
    raw = np.ascontiguousarray(xf.raw("l.0.attn.q.weight"))
    with pytest.raises(L.XhError):  # one byte short of whole blocks
        gm.upload(L.WQ, 0, L.Q8_0, raw[:-1])
    gm.upload(L.WQ, 0, L.Q8_0, raw)
    gm.close()


@pytest.mark.parametrize("name", ["tiny_mistral_q8_0", "tiny_mistral_q4_0", "small_llama_q8_0"])
@pytest.mark.parametrize("batched", [1, 3, 0])
def test_block_prompt_passes(name, batched):
    """A 100-token prompt through the batched path on gguf blocks (XH_OPT_PREFILL 1: the blocks'
    exact f16 hi + lo images through gemm16.h, one pass; 3: the f32-input MFMA kernel decoding the
    blocks in registers, a full 64-token pass + 36) and the token loop (0) vs the oracle's HYDRATE
    loop: last logits, every K/V row; then the perplexity path over 80 tokens (lm_head GEMM over
    block rows)."""
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf, context=256)
    gm.set_option(L.OPT_PREFILL, batched)
    om = O.OracleModel.from_xalm(xf, context=256)
    toks = [1] + [3 + (i * 41) % (gm.config.vocab_size - 3) for i in range(99)]
    st = InferenceState(gm.config)
    gm.prefill(toks, 0, st)
    for pos, tok in enumerate(toks):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
    check(st.logits(), om.logits(), name, "prefill" if batched else "loop")
    for layer in range(gm.config.n_layers):
        for which in (0, 1):
            a = gm.kv_read(layer, which, 0, len(toks)).view(np.float16).astype(np.float32)
            b = om.kv(layer, which)[:len(toks)].view(np.float16).astype(np.float32)
            assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), (layer, which)
    gm.close()
    gm2 = Model.from_xalm(xf, context=256)
    gm2.set_option(L.OPT_PREFILL, batched)
    om2 = O.OracleModel.from_xalm(xf, context=256)
    got = gm2.token_probs(toks[:80])
    for pos in range(79):
        om2.forward(toks[pos], pos)
        lg = om2.logits()
        ref = O.sample_prob(lg, toks[pos + 1])
        if ref < 1e-30:
            assert got[pos] < 1e-30
            continue
        check_logp(float(abs(np.log(got[pos]) - np.log(ref))), lg, name, pos)


@pytest.mark.parametrize("name", ["tiny_mistral_q4_0", "tiny_mistral_q8_0"])
def test_block_multi_pass_prefill(name):
    """2200 tokens = a full 2048-token gemm16.h pass over the hi / lo block images and a 152-token
    one attending over the first pass's K/V rows, vs the oracle's token loop."""
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf, context=4096)
    om = O.OracleModel.from_xalm(xf, context=4096)
    toks = [1] + [3 + (i * 41) % (gm.config.vocab_size - 3) for i in range(2199)]
    st = InferenceState(gm.config)
    gm.prefill(toks, 0, st)
    for pos, tok in enumerate(toks):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
    check(st.logits(), om.logits(), name, "prefill")
    for layer in range(gm.config.n_layers):
        a = gm.kv_read(layer, 1, 0, len(toks)).view(np.float16).astype(np.float32)
        b = om.kv(layer, 1)[:len(toks)].view(np.float16).astype(np.float32)
        assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), layer
