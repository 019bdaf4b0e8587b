"""Pin the CPU oracle (oracle/xalm_oracle.c) before trusting it as the checker.

* against HuggingFace logits on .xalm fixtures written by the reference's own convert.py
  (tests/golden/make_fixtures.py);
* element decoders against numpy / torch for every code;
* sampler quirks of src/sampler.cpp.
"""
import os

import numpy as np
import pytest

from conftest import fixture_path
from oracle import oracle as O
from xalm_amd import _lib as L
from xalm_amd.xalm_file import XalmFile


@pytest.mark.parametrize("name,t", [("tiny_mistral", "f16"), ("tiny_mistral", "bf16"), ("tiny_mistral", "f32"),
                                    ("small_llama", "f16")])
def test_oracle_matches_hf(name, t):
    g = np.load(fixture_path(f"hf_logits_{name}.npz"))
    toks, hf, hf16 = g["tokens"], g["logits"], g["logits_f16kv"]
    m = O.OracleModel.from_xalm(XalmFile(fixture_path(f"{name}_{t}.xalm")))
    for pos, tok in enumerate(toks):
        m.forward(tok, pos, L.OUTPUT_LOGITS)
        lg = m.logits()
        scale = max(1.0, float(np.abs(hf16[pos]).max()))
        # HF with the reference's fp16 KV rounding: summation-order differences only
        assert np.abs(lg - hf16[pos]).max() <= 5e-4 * scale, pos
        # plain HF (fp32 KV): the fp16 KV cache is the dominant gap (4.8e-4)
        assert np.abs(lg - hf[pos]).max() <= 5e-3 * scale, pos
        assert lg.argmax() == hf[pos].argmax()
    if name == "tiny_mistral":
        assert max(np.abs(m.logits() - hf[-1]).max(), 0) < 1e-3


@pytest.mark.parametrize("t", ["f8_e4m3", "f8_e5m2"])
def test_oracle_fp8_fixture_runs_and_tracks_hf(t):
    g = np.load(fixture_path("hf_logits_tiny_mistral.npz"))
    m = O.OracleModel.from_xalm(XalmFile(fixture_path(f"tiny_mistral_{t}.xalm")))
    errs = []
    for pos, tok in enumerate(g["tokens"]):
        m.forward(tok, pos, L.OUTPUT_LOGITS)
        errs.append(np.abs(m.logits() - g["logits"][pos]).max())
    # fp8 quantisation error only (HF ran the bf16 weights)
    assert np.isfinite(errs).all() and max(errs) < 0.5


def test_f16_to_f32_all_codes():
    codes = np.arange(65536, dtype=np.uint16)
    ref = codes.view(np.float16).astype(np.float32)
    got = np.array([O.f16_to_f32(int(c)) for c in codes[::7]], dtype=np.float32)
    r = ref[::7]
    nan = np.isnan(r)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), r[~nan].view(np.uint32))


def test_f32_to_f16_round_to_nearest_even():
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.standard_normal(3000).astype(np.float32) * s for s in (1e-7, 1e-5, 1e-3, 1, 1e3, 6e4)])
    specials = np.array([0.0, -0.0, 65504.0, 65519.99, 65520.0, 1e9, -1e9, np.inf, -np.inf,
                         5.960464477539063e-08, 2.980232238769531e-08, 2.9802326e-08, 6.1035156e-05,
                         1.0 + 2 ** -11, 1.0 + 3 * 2 ** -11], dtype=np.float32)
    vals = np.concatenate([vals, specials])
    ref = vals.astype(np.float16).view(np.uint16)
    got = np.array([O.f32_to_f16(float(v)) for v in vals], dtype=np.uint16)
    assert np.array_equal(got, ref)


def test_fp8_decode_matches_torch_for_finite_codes():
    torch = pytest.importorskip("torch")
    codes = np.arange(256, dtype=np.uint8)
    for dt, tdt, nan_codes in ((L.F8_E4M3, torch.float8_e4m3fn, {0x7F: 480.0, 0xFF: -480.0}),
                               (L.F8_E5M2, torch.float8_e5m2, None)):
        ref = torch.from_numpy(codes.copy()).view(tdt).float().numpy()
        got = np.array([O.decode(dt, codes, i) for i in range(256)], dtype=np.float32)
        fin = np.isfinite(ref)
        assert np.array_equal(got[fin], ref[fin])
        if nan_codes:  # f8_t::to_float gives finite values for the NaN codes (src/types.h:302-314)
            for c, v in nan_codes.items():
                assert got[c] == v
        else:  # e5m2 Inf/NaN codes: exponent field 31 decodes finite (0x7C -> 65536)
            assert got[0x7C] == 65536.0 and np.isfinite(got).all()


def test_q8_and_bf16_decode():
    q = np.arange(-128, 128, dtype=np.int8)
    got = np.array([O.decode(L.Q8, q, i) for i in range(256)], dtype=np.float32)
    assert np.array_equal(got, np.float32(1.0 / 100.0) * q.astype(np.float32))
    b = np.array([0x3F80, 0xC000, 0x0001, 0x7F7F], dtype=np.uint16)
    got = np.array([O.decode(L.BF16, b, i) for i in range(4)], dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), b.astype(np.uint32) << 16)


def test_sampler_quirks():
    # max starts at FLT_MIN: all-negative logits give token 0 (src/sampler.cpp:22)
    assert O.sample_argmax(np.array([-3.0, -1.0, -2.0], dtype=np.float32)) == 0
    # first index of the maximum wins
    assert O.sample_argmax(np.array([0.5, 2.0, 2.0, 1.0], dtype=np.float32)) == 1
    lg = np.array([1.0, 2.0, 3.0], dtype=np.float32)
    p = np.exp(lg - 3.0) / np.exp(lg - 3.0).sum()
    assert abs(O.sample_prob(lg, 2) - p[2]) < 1e-6


def test_matmul_oracle_vs_numpy():
    rng = np.random.default_rng(1)
    n, d = 256, 96
    x = rng.standard_normal(n).astype(np.float32)
    w = (rng.standard_normal((d, n)) * 0.05).astype(np.float16)
    got = O.matmul(x, w.view(np.uint16), L.F16, n, d)
    ref = w.astype(np.float64) @ x.astype(np.float64)
    assert np.abs(got - ref).max() < 1e-4


def test_active_bytes_formula():
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    m = O.OracleModel.from_xalm(xf)
    c = xf.config()
    per_layer = (2 * c.dim * 2 + (c.n_heads + 2 * c.n_kv_heads) * c.head_dim * c.dim * 2 +
                 c.n_heads * c.head_dim * c.dim * 2 + 3 * c.dim * c.hidden_dim * 2)
    for pos in (0, 10, 1000):
        kv_len = min(c.max_seq_len, pos + 1)
        exp = c.dim * 2 + c.dim * 2 + c.vocab_size * c.dim * 2 + c.n_layers * (
            per_layer + 2 * kv_len * c.n_kv_heads * c.head_dim * 2)
        assert m.active_bytes(pos) == exp


def test_oracle_ring_mode_runs_past_context():
    # -T smaller than the sequence: ring buffer + 2 attention sinks (src/infer.cpp:608-613, 416-431)
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    m = O.OracleModel.from_xalm(xf, context=16)
    for pos in range(40):
        m.forward(3 + (pos * 7) % 200, pos, L.OUTPUT_LOGITS)
        assert np.isfinite(m.logits()).all()


@pytest.mark.parametrize("name,t", [("tiny_mistral", "f16"), ("small_llama", "f16"), ("tiny_mistral", "f8_e4m3"),
                                    ("tiny_mistral", "q4_0")])
def test_oracle_f64_evaluation(name, t):
    """xo_set_precision(m, 1) evaluates the same algorithm in double (the yardstick of
    tests/test_parity_full_gpu.py): on the fixtures it stays within the north-star bar of the f32
    evaluation at every position, the first layer's fp16 K rows agree to one fp16 ulp, and the f32 evaluation
    of a fresh model is unaffected (bitwise)."""
    xf = XalmFile(fixture_path(f"{name}_{t}.xalm"))
    m32, m64, again = (O.OracleModel.from_xalm(xf) for _ in range(3))
    m64.set_precision(1)
    assert m64.set_precision is not None and O._load().xo_precision(m64.m) == 1
    toks = [1] + [3 + (i * 37) % 280 for i in range(23)]
    for pos, tok in enumerate(toks):
        m32.forward(tok, pos)
        m64.forward(tok, pos)
        again.forward(tok, pos)
        a, b = m32.logits(), m64.logits()
        assert np.abs(a - b).max() <= 1e-3 * max(1.0, float(np.abs(b).max())), pos
        assert np.array_equal(a.view(np.uint32), again.logits().view(np.uint32))
    for layer in range(xf.config().n_layers):
        ka = m32.kv(layer, 0)[:len(toks)].view(np.float16).astype(np.float32)
        kb = m64.kv(layer, 0)[:len(toks)].view(np.float16).astype(np.float32)
        if layer == 0:  # one rounding apart at most
            assert np.all(np.abs(ka - kb) <= np.abs(kb) * 2.0 ** -10 + 2.0 ** -24)
        else:  # after a layer of differently rounded activations: the GPU tests' K/V bar
            assert np.abs(ka - kb).max() <= 2e-3 * max(1.0, float(np.abs(kb).max())), layer


_ISA_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
rng = np.random.default_rng(3)
out = {}
for dt in (2, 6, 7, 20, 21):
    n, d = 4096 + 40, 48
    if dt == 2:
        w = rng.standard_normal((d, n)).astype(np.float16).view(np.uint16)
    elif dt in (20, 21):  # gguf Q8_0 / Q4_0 blocks of the converter's quantizer (n % 32 == 0)
        n = 4096 + 64
        w = O.quantize_gq(dt, (0.02 * rng.standard_normal((d, n))).astype(np.float32))
    else:
        w = rng.integers(0, 256, (d, n), dtype=np.uint8)
    x = rng.standard_normal(n).astype(np.float32)
    o = np.zeros(d, np.float32)
    O._load().xo_matmul(O._p(o), O._p(x), O._p(np.ascontiguousarray(w)), dt, n, d)
    out[dt] = o.view(np.uint32).tolist()
print(O.isa(), out)
"""


def test_lanes_order_same_bits_on_every_isa():
    """The lanes-order matvec (f16, e4m3, e5m2, gguf Q8_0 / Q4_0) picks AVX-512 or AVX2 at run time
    (-march=native); both forms must give the same bits, so the timed CPU
    baseline and the parity tests' f32 evaluation are one algorithm on any host."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    runs = []
    for env_extra in ({}, {"XO_NO_AVX512": "1"}):
        env = dict(os.environ, **env_extra)
        r = subprocess.run([sys.executable, "-c", _ISA_SCRIPT, root], capture_output=True, text=True, env=env,
                           timeout=120, check=True)
        isa, res = r.stdout.strip().split(" ", 1)
        runs.append((int(isa), res))
    assert runs[1][0] == 1
    assert runs[0][1] == runs[1][1]


@pytest.mark.parametrize("dt", [L.Q8_0, L.Q4_0])
def test_gguf_matvec_orders(dt):
    """gguf matvec (quants.py blocks dequantized exactly, then the reference's f32 row loop):
    the vectorised lanes order (default) and the sequential order agree with a float64 sum of
    the dequantized products to f32 accuracy; the sequential order is the scalar loop."""
    rng = np.random.default_rng(5)
    n, d = 4096, 64
    vals = (0.02 * rng.standard_normal((d, n))).astype(np.float32)
    w = O.quantize_gq(dt, vals)
    x = rng.standard_normal(n).astype(np.float32)
    deq = np.array([[O.decode_row(dt, w, r, n, i) for i in range(n)] for r in range(4)], np.float64)
    ref = deq @ x.astype(np.float64)
    mag = np.abs(deq) @ np.abs(x.astype(np.float64))
    outs = []
    for order in (0, 1):
        O.set_matmul_order(order)
        try:
            outs.append(O.matmul(x, w, dt, n, d))
        finally:
            O.set_matmul_order(0)
    for o in outs:
        assert np.all(np.abs(o[:4] - ref) <= 1e-5 * mag + 1e-7)
    assert not np.array_equal(outs[0], outs[1])  # two summation orders, both valid readings
