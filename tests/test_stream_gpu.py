"""Stream engine (xh_set_engine(2), xalm_amd/csrc/stream.h) vs the CPU oracle.

The stream kernel needs rows of whole 1 KiB K-steps (f16: dim, q_dim, hidden multiples of
512), so these tests run synthetic models (include/xalm_synth.h weights, the same bytes in the
oracle) instead of the tiny converter fixtures.  Bars as tests/test_forward_gpu.py: logits
within 1e-3 * max(1, max|logit|) of the oracle at every checked position; K/V rows within the
fp16 rounding of the oracle's rows; greedy tokens equal to the oracle's argmax wherever the
top two logits are not a near-tie.
"""
import numpy as np
import pytest

import bench
from oracle import oracle as O
from xalm_amd import _lib as L
from xalm_amd.model import InferenceState, Model

pytestmark = pytest.mark.gpu

BASE = dict(dim=1024, hidden=2048, layers=2, heads=8, kv_heads=2, head_dim=128, vocab=1000, msl=512,
            theta=1e6, wdt=L.F16, edt=L.F16, cdt=L.F16)


def tol(ref):
    return 1e-3 * max(1.0, float(np.abs(ref).max()))


def pair(**kw):
    w = dict(BASE, **kw)
    c = bench.make_config(w)
    gm, om = Model(c), O.OracleModel(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
        rows, cols = bench.tensor_shape(c, kind)
        om.set_tensor(kind, layer, dt, O.synthetic(rows, cols, dt, seed, mean, std))
    gm.set_engine(2)
    assert gm.engine == 2
    return gm, om, c


def toks_for(c, n, mul=37):
    return [1] + [3 + (i * mul) % (c.vocab_size - 3) for i in range(n - 1)]


@pytest.mark.parametrize("case", ["f16", "bf16", "f32", "f8_e4m3", "f8_e5m2", "hd64"])
def test_stream_forward_matches_oracle(case):
    kw = {"f16": {}, "bf16": dict(wdt=L.BF16, edt=L.BF16, cdt=L.BF16), "f32": dict(wdt=L.F32, edt=L.F32, cdt=L.F32),
          "f8_e4m3": dict(wdt=L.F8_E4M3, edt=L.BF16, cdt=L.BF16),
          "f8_e5m2": dict(wdt=L.F8_E5M2, edt=L.BF16, cdt=L.BF16),
          "hd64": dict(heads=16, kv_heads=4, head_dim=64)}[case]
    gm, om, c = pair(**kw)
    st = InferenceState(c)
    for pos, tok in enumerate(toks_for(c, 12)):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        ref = om.logits()
        assert np.isfinite(st.logits()).all()
        err = float(np.abs(st.logits() - ref).max())
        assert err <= tol(ref), (case, pos, err)
    # the K/V rows the stream kernel wrote: fp16 of values within the fp32 tolerance
    kv_dim = c.n_kv_heads * c.head_dim
    for layer in range(c.n_layers):
        for which in (0, 1):
            got = gm.kv_read(layer, which, 0, 12).view(np.float16).astype(np.float32)
            exp = om.kv(layer, which)[:12].view(np.float16).astype(np.float32).reshape(got.shape)
            assert got.shape == (12, kv_dim)
            assert np.abs(got - exp).max() <= 2e-3 * max(1.0, np.abs(exp).max()), (case, layer, which)
    gm.close()
    om.close()


def test_stream_hydrate_then_decode_teacher_forced():
    # one launch hydrates the prompt (HYDRATE mode for all but the last token), a second decodes
    # 24 greedy tokens on the device; the oracle replays the same tokens
    gm, om, c = pair()
    gm.set_option(L.OPT_PREFILL, 0)  # the prompt goes through the stream kernel's token loop
    st = InferenceState(c)
    prompt = toks_for(c, 9, mul=53)
    gm.prefill(prompt, 0, st)
    for pos, tok in enumerate(prompt):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(prompt) - 1 else L.HYDRATE_KV_CACHE)
    assert np.abs(st.logits() - om.logits()).max() <= tol(om.logits())
    toks = gm.decode_greedy(len(prompt), 24)
    assert len(toks) == 24
    pos = len(prompt)
    for t in toks:
        lg = om.logits()
        top2 = np.sort(lg)[-2:]
        if top2[1] - top2[0] > 1e-3:
            assert t == O.sample_argmax(lg)
        om.forward(t, pos)
        pos += 1
    gm.get_logits(st)
    assert np.abs(st.logits() - om.logits()).max() <= tol(om.logits())
    gm.close()
    om.close()


def test_stream_equals_graph_engine_tokens():
    # 64 greedy tokens: the stream engine's tokens equal the graph engine's
    outs = []
    for engine in (0, 2):
        gm, om, c = pair()
        gm.set_engine(engine)
        st = InferenceState(c)
        gm.prefill([1, 7, 99], 0, st)
        toks = gm.decode_greedy(3, 64)
        gm.get_logits(st)
        outs.append((toks, st.logits().copy()))
        gm.close()
        om.close()
    assert outs[0][0] == outs[1][0]
    assert np.abs(outs[0][1] - outs[1][1]).max() <= tol(outs[0][1])


def test_stream_decode_stops_on_eos():
    gm, om, c = pair()
    st = InferenceState(c)
    gm.forward(st, 1, 0)
    first = gm.decode_greedy(1, 4)
    gm.reset()
    gm.forward(st, 1, 0)
    got = gm.decode_greedy(1, 10, stop=(first[2], -1))
    assert got == first[:3]
    # and the context still works after the early exit (the loader left cleanly)
    gm.reset()
    gm.forward(st, 1, 0)
    om.forward(1, 0)
    assert np.abs(st.logits() - om.logits()).max() <= tol(om.logits())
    gm.close()
    om.close()


@pytest.mark.parametrize("history", [0, 300, 900])
def test_stream_multi_split_attention(history):
    # kv_len > the split length: several (head, split) items per KV head, merged by the last
    # split; a filled KV history makes long rows without a long oracle loop
    gm, om, c = pair(msl=1024)
    kv_dim = c.n_kv_heads * c.head_dim
    for layer in range(c.n_layers):
        for which in (0, 1):
            if history:
                seed = 900 + 2 * layer + which
                gm.kv_fill_synthetic(layer, which, 0, history, seed, 1.0)
                om.set_kv(layer, which, 0, O.synthetic(history, kv_dim, L.F16, seed, 0.0, 1.0))
    st = InferenceState(c)
    for i, tok in enumerate(toks_for(c, 6 if history else 160, mul=29)):
        pos = history + i
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        if history or i % 40 == 39:
            ref = om.logits()
            assert np.abs(st.logits() - ref).max() <= tol(ref), (history, pos)
    gm.close()
    om.close()


def test_stream_ring_buffer_and_sinks():
    # -T 64 with 90 tokens: the KV ring wraps, the two sink rows are re-roped every step
    gm, om, c = pair(msl=64)
    st = InferenceState(c)
    for pos, tok in enumerate(toks_for(c, 90, mul=31)):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        if pos >= 60:
            ref = om.logits()
            assert np.abs(st.logits() - ref).max() <= tol(ref), pos
    gm.close()
    om.close()


def test_stream_engine_refuses_unaligned_rows():
    # dim 256 f16 = 512-byte rows: not whole 1 KiB K-steps -> XH_E_INVALID, engine unchanged
    w = dict(BASE, dim=256, hidden=512, heads=2, kv_heads=1)
    gm = Model(bench.make_config(w))
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
    with pytest.raises(L.XhError):
        gm.set_engine(2)
    assert gm.engine == 0
    gm.close()
