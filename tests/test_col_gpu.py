"""Column-form attention + Wo (xalm_amd/csrc/attn_col.h, XH_OPT_COL_KV_MAX) vs the CPU oracle.

Each workgroup of the column form computes one KV head's attention itself and multiplies it by
its slice of Wo's columns; the W1/W3 launch's rmsnorm prologue sums the per-head partials
(gemv.h PRO_RMSNORM_P).  Synthetic models (include/xalm_synth.h weights, the same bytes in the
oracle) at dims that take both prologue forms (dim 2048 f16: x held in registers, the PF
prologue; dim 1024: the staged prologue).  Bars as tests/test_forward_gpu.py: logits within
1e-3 * max(1, max|logit|) of the oracle; greedy tokens equal the oracle's argmax wherever the
top two logits are not a near-tie.  tests/test_forward_gpu.py runs the converter fixtures
through it too (engine "graph_col").
"""
import numpy as np
import pytest

import bench
from oracle import oracle as O
from xalm_amd import _lib as L
from xalm_amd.model import InferenceState, Model

pytestmark = pytest.mark.gpu

BASE = dict(dim=2048, hidden=1024, layers=2, heads=16, kv_heads=4, head_dim=128, vocab=1000, msl=512,
            theta=1e6, wdt=L.F16, edt=L.F16, cdt=L.F16)


def tol(ref):
    return 1e-3 * max(1.0, float(np.abs(ref).max()))


def pair(col_max=256, **kw):
    w = dict(BASE, **kw)
    c = bench.make_config(w)
    gm, om = Model(c), O.OracleModel(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
        rows, cols = bench.tensor_shape(c, kind)
        om.set_tensor(kind, layer, dt, O.synthetic(rows, cols, dt, seed, mean, std))
    gm.set_option(L.OPT_COL_KV_MAX, col_max)
    return gm, om, c


def toks_for(c, n, mul=37):
    return [1] + [3 + (i * mul) % (c.vocab_size - 3) for i in range(n - 1)]


CASES = {"f16": {}, "f16_d1024": dict(dim=1024), "bf16": dict(wdt=L.BF16, edt=L.BF16, cdt=L.BF16),
         "f8_e4m3": dict(wdt=L.F8_E4M3, edt=L.BF16, cdt=L.BF16), "f8_e5m2": dict(wdt=L.F8_E5M2, edt=L.BF16, cdt=L.BF16),
         "hd64": dict(heads=32, kv_heads=8, head_dim=64), "qpk8": dict(heads=16, kv_heads=2, head_dim=64)}


@pytest.mark.parametrize("case", list(CASES))
def test_col_forward_matches_oracle(case):
    gm, om, c = pair(**CASES[case])
    qpk = c.n_heads // c.n_kv_heads
    supported = (c.head_dim, qpk) in ((128, 4), (64, 4), (16, 2))
    assert gm.get_option(L.OPT_COL_KV_MAX) == (256 if supported else 0)
    st = InferenceState(c)
    n = 12
    for pos, tok in enumerate(toks_for(c, n)):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        ref = om.logits()
        assert np.isfinite(st.logits()).all()
        err = float(np.abs(st.logits() - ref).max())
        assert err <= tol(ref), (case, pos, err)
    for layer in range(c.n_layers):
        for which in (0, 1):
            got = gm.kv_read(layer, which, 0, n).view(np.float16).astype(np.float32)
            exp = om.kv(layer, which)[:n].view(np.float16).astype(np.float32).reshape(got.shape)
            assert np.abs(got - exp).max() <= 2e-3 * max(1.0, np.abs(exp).max()), (case, layer, which)
    gm.close()
    om.close()


def test_col_f32_wo_takes_the_split_form():
    # f32 Wo at head_dim 128 x 4 q heads = 128 chunks of 16 B per head slice: not instantiated
    gm, om, c = pair(wdt=L.F32, edt=L.F32, cdt=L.F32)
    assert gm.get_option(L.OPT_COL_KV_MAX) == 0
    st = InferenceState(c)
    for pos, tok in enumerate(toks_for(c, 4)):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
    assert np.abs(st.logits() - om.logits()).max() <= tol(om.logits())
    gm.close()
    om.close()


def test_col_equals_split_form_tokens():
    # 48 greedy tokens with the column form on (every step) and off: the same tokens, logits
    # within the bar
    outs = []
    for col_max in (256, 0):
        gm, om, c = pair(col_max=col_max)
        st = InferenceState(c)
        gm.prefill(toks_for(c, 5, mul=41), 0, st)
        toks = gm.decode_greedy(5, 48)
        gm.get_logits(st)
        outs.append((toks, st.logits().copy()))
        gm.close()
        om.close()
    assert outs[0][0] == outs[1][0]
    assert np.abs(outs[0][1] - outs[1][1]).max() <= tol(outs[1][1])


def test_col_threshold_crossing_in_decode_loop():
    # bound 20: the device loop switches graphs at history 21; teacher-forced oracle replay
    gm, om, c = pair(col_max=20)
    st = InferenceState(c)
    prompt = toks_for(c, 10, mul=53)
    gm.prefill(prompt, 0, st)
    for pos, tok in enumerate(prompt):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(prompt) - 1 else L.HYDRATE_KV_CACHE)
    toks = gm.decode_greedy(len(prompt), 24)
    pos = len(prompt)
    for t in toks:
        lg = om.logits()
        top2 = np.sort(lg)[-2:]
        if top2[1] - top2[0] > 1e-3:
            assert t == O.sample_argmax(lg), pos
        om.forward(t, pos)
        pos += 1
    gm.get_logits(st)
    assert np.abs(st.logits() - om.logits()).max() <= tol(om.logits())
    gm.close()
    om.close()


@pytest.mark.parametrize("history", [60, 130, 250])
def test_col_long_history(history):
    # filled K/V histories up to the column form's 256-slot bound (every row of the head in
    # LDS); the same rows in the oracle
    gm, om, c = pair()
    kv_dim = c.n_kv_heads * c.head_dim
    for layer in range(c.n_layers):
        for which in (0, 1):
            seed = 700 + 2 * layer + which
            gm.kv_fill_synthetic(layer, which, 0, history, seed, 1.0)
            om.set_kv(layer, which, 0, O.synthetic(history, kv_dim, L.F16, seed, 0.0, 1.0))
    st = InferenceState(c)
    for i, tok in enumerate(toks_for(c, 6, mul=29)):
        pos = history + i
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        ref = om.logits()
        assert np.abs(st.logits() - ref).max() <= tol(ref), (history, pos)
    gm.close()
    om.close()


def test_col_option_bounds():
    gm, om, c = pair(col_max=0)
    assert gm.get_option(L.OPT_COL_KV_MAX) == 0
    with pytest.raises(L.XhError):
        gm.set_option(L.OPT_COL_KV_MAX, 257)
    gm.set_option(L.OPT_FUSE_ATTN_WO, 0)
    gm.set_option(L.OPT_COL_KV_MAX, 200)
    assert gm.get_option(L.OPT_COL_KV_MAX) == 0  # only at fusion level 1
    gm.set_option(L.OPT_FUSE_ATTN_WO, 1)
    assert gm.get_option(L.OPT_COL_KV_MAX) == 200
    gm.close()
    om.close()
