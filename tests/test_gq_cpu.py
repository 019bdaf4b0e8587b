"""gguf block formats (Q8_0 / Q4_0): the oracle and the shared quantizer vs the
reference's quants.py, bit for bit.

tests/golden/gq_golden.npz holds quants.py ``quantize`` bytes and ``dequantize`` floats of
seeded rows and edge rows (tests/golden/make_gq_fixtures.py).  The oracle's decode
(oracle/xalm_oracle.c xo_decode_row, restating quants.py Q8_0 :448-454 / Q4_0 :302-311) must
reproduce the floats exactly, and the quantizer in include/xalm_synth.h (used by the
oracle's and the device's synthetic weights) must reproduce the bytes exactly.
"""
import numpy as np
import pytest

from conftest import fixture_path
from oracle import oracle as O
from xalm_amd import _lib as L
from xalm_amd.xalm_file import XalmFile

G = np.load(fixture_path("gq_golden.npz"))
TYPES = {"q8_0": L.Q8_0, "q4_0": L.Q4_0}


@pytest.mark.parametrize("name", list(TYPES))
def test_quantizer_matches_quants_py(name):
    got = O.quantize_gq(TYPES[name], G["inputs"])
    assert got.shape == G[name].shape
    assert np.array_equal(got, G[name]), np.argwhere(got != G[name])[:5]


@pytest.mark.parametrize("name", list(TYPES))
def test_oracle_decode_matches_quants_py(name):
    q, deq = G[name], G[name + "_deq"]
    rows, n = deq.shape
    got = np.array([[O.decode_row(TYPES[name], q, r, n, i) for i in range(n)] for r in range(rows)], np.float32)
    assert np.array_equal(got.view(np.uint32), deq.view(np.uint32))


@pytest.mark.parametrize("name", list(TYPES))
def test_oracle_matmul_uses_the_dequantized_rows(name):
    # xo_matmul over blocks == the reference row loop over quants.py's dequantized floats: the
    # sequential order against that loop in float32, the default lanes order (blocks dequantized
    # 32 at a time, 8-wide FMA lanes) against a float64 sum within f32 accumulation error
    q, deq = G[name], G[name + "_deq"]
    x = np.random.default_rng(5).normal(0, 1, deq.shape[1]).astype(np.float32)
    lib = O._load()
    outs = {}
    for order in (1, 0):
        out = np.zeros(deq.shape[0], np.float32)
        O.set_matmul_order(order)
        try:
            lib.xo_matmul(O._p(out), O._p(x), O._p(np.ascontiguousarray(q)), TYPES[name], deq.shape[1], deq.shape[0])
        finally:
            O.set_matmul_order(0)
        outs[order] = out
    ref = np.zeros_like(outs[1])
    for r in range(deq.shape[0]):
        v = np.float32(0)
        for j in range(deq.shape[1]):
            v = np.float32(v + deq[r, j] * x[j])
        ref[r] = v
    assert np.abs(outs[1] - ref).max() <= 1e-6 * max(1.0, float(np.abs(ref).max()))
    d64 = deq.astype(np.float64)
    exact = d64 @ x.astype(np.float64)
    mag = np.abs(d64) @ np.abs(x.astype(np.float64))
    assert np.all(np.abs(outs[0] - exact) <= 2e-6 * mag + 1e-7)


@pytest.mark.parametrize("name", ["tiny_mistral_q8_0", "tiny_mistral_q4_0"])
def test_oracle_forward_on_converter_blocks(name):
    # the converter's block files run through the oracle; logits track the f16 conversion of
    # the same checkpoint within the quantization error (Q4_0 coarser)
    toks = [1, 5, 77, 200, 9, 31]
    outs = []
    for fx in (name, "tiny_mistral_f16"):
        xf = XalmFile(fixture_path(fx + ".xalm"))
        om = O.OracleModel.from_xalm(xf)
        for pos, t in enumerate(toks):
            om.forward(t, pos)
        outs.append(om.logits())
        om.close()
    assert np.isfinite(outs[0]).all()
    rel = np.abs(outs[0] - outs[1]).max() / np.abs(outs[1]).max()
    assert rel < (0.05 if "q8_0" in name else 0.3), rel


def test_synthetic_blocks_shape_and_determinism():
    a = O.synthetic(3, 64, L.Q8_0, 11, 0.0, 0.02)
    b = O.synthetic(3, 64, L.Q8_0, 11, 0.0, 0.02)
    assert a.shape == (3, 68) and np.array_equal(a, b)
    c = O.synthetic(3, 64, L.Q4_0, 11, 0.0, 0.02)
    assert c.shape == (3, 36)
