"""Whole-forward parity: Model.forward on the HIP path vs the CPU oracle (and HF goldens).

Fixtures are .xalm files written by the reference's convert.py (tests/golden/).
Bars (tests/bars.py): on the fixtures 8x the measured GPU-vs-oracle envelope of that fixture
and path (tests/golden/error_envelope.json), capped by the north-star bar, 1e-3 max-abs stated
relative to the logit scale above 1 (small_llama's logits reach |93|); on synthetic models the
north-star bar.
"""
import numpy as np
import pytest

from bars import bar, check, check_logp
from conftest import fixture_path
from oracle import oracle as O
from xalm_amd import _lib as L
from xalm_amd.model import InferenceState, Model
from xalm_amd.xalm_file import XalmFile

pytestmark = pytest.mark.gpu

FIXTURES = ["tiny_mistral_f16", "tiny_mistral_bf16", "tiny_mistral_f32", "tiny_mistral_f8_e4m3",
            "tiny_mistral_f8_e5m2", "small_llama_f16"]


# launch structures of the hipGraph step: "graph": qkv, then attention + Wo in one launch
# (attn_wo.h, the default); "graph_split": attention and Wo as two launches
ENGINES = ["graph", "graph_split"]
FUSE = {"graph": 1, "graph_split": 0}


def configure(gm, engine):
    gm.set_option(L.OPT_FUSE_ATTN_WO, FUSE[engine])
    assert gm.get_option(L.OPT_FUSE_ATTN_WO) == FUSE[engine]


def run_pair(name, tokens, context=0, graphs=True, modes=None, engine="graph"):
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf, context=context)
    gm.set_graphs(graphs)
    configure(gm, engine)
    om = O.OracleModel.from_xalm(xf, context=context)
    st = InferenceState(gm.config)
    worst = 0.0
    for pos, tok in enumerate(tokens):
        mode = L.OUTPUT_LOGITS if modes is None else modes[pos]
        gm.forward(st, tok, pos, mode)
        om.forward(tok, pos, mode)
        if mode == L.OUTPUT_LOGITS:
            ref = om.logits()
            err = check(st.logits(), ref, name, "loop", pos)
            worst = max(worst, err / bar(ref, name))
    return gm, om, worst


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("name", FIXTURES)
def test_forward_matches_oracle(name, engine):
    g = np.load(fixture_path("hf_logits_%s.npz" % name.rsplit("_", 1)[0].replace("_f8", "")))
    toks = [int(t) for t in g["tokens"]]
    gm, om, worst = run_pair(name, toks, engine=engine)
    # KV rings equal the oracle's up to fp16 rounding: both round to nearest-even, but the fp32
    # values differ in the last bits (summation order, amplified through the layers), so values
    # near a rounding boundary land an ulp apart.  Layer 0 (inputs identical up to rmsnorm
    # order): <= 1 fp16 ulp of the element; every layer: <= 1e-3 of the ring's max |value|;
    # most elements bit-identical (DPP reduction order: up to ~10 % flip in the tiny model).
    c = gm.config
    n = len(toks)
    for layer in range(c.n_layers):
        for which in (0, 1):
            a = gm.kv_read(layer, which, 0, n).view(np.float16).astype(np.float32)
            b = om.kv(layer, which)[:n].view(np.float16).astype(np.float32)
            d = np.abs(a - b)
            assert (d > 0).mean() < 0.25, (layer, which, (d > 0).mean())
            assert d.max() <= 1e-3 * np.abs(b).max(), (layer, which, float(d.max()))
            if layer == 0:
                assert np.all(d <= np.abs(b) * 2.0 ** -10 + 2.0 ** -24), (which, float(d.max()))


@pytest.mark.parametrize("name", ["tiny_mistral_f16", "small_llama_f16"])
def test_forward_matches_hf(name):
    base = name.rsplit("_", 1)[0]
    g = np.load(fixture_path(f"hf_logits_{base}.npz"))
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf)
    st = InferenceState(gm.config)
    for pos, tok in enumerate(g["tokens"]):
        gm.forward(st, int(tok), pos)
        ref = g["logits_f16kv"][pos]
        assert np.abs(st.logits() - ref).max() <= 5e-4 * max(1.0, np.abs(ref).max())
        assert st.logits().argmax() == g["logits"][pos].argmax()


@pytest.mark.parametrize("engine", ENGINES)
def test_ring_buffer_and_sinks(engine):
    # -T 16 with 48 tokens: kv_sink=2, ring wrap, sink re-rotation every step (src/infer.cpp:608-613, 421-431)
    toks = [1] + [3 + (i * 37) % 290 for i in range(47)]
    gm, om, _ = run_pair("tiny_mistral_f16", toks, context=16, engine=engine)
    for layer in range(gm.config.n_layers):
        a = gm.kv_read(layer, 0, 0, 16).view(np.float16).astype(np.float32)
        b = om.kv(layer, 0)[:16].view(np.float16).astype(np.float32)
        assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max())


@pytest.mark.parametrize("engine", ENGINES)
def test_ring_buffer_head_dim_128(engine):
    toks = [1] + [3 + (i * 53) % 310 for i in range(39)]
    run_pair("small_llama_f16", toks, context=24, engine=engine)


@pytest.mark.parametrize("engine", ENGINES)
def test_hydrate_mode_then_logits(engine):
    toks = [1] + [3 + (i * 11) % 290 for i in range(15)]
    modes = [L.HYDRATE_KV_CACHE] * (len(toks) - 1) + [L.OUTPUT_LOGITS]
    run_pair("tiny_mistral_f16", toks, modes=modes, engine=engine)


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("name,context", [("tiny_mistral_f16", 16), ("small_llama_f16", 0),
                                          ("tiny_mistral_f8_e4m3", 0)])
def test_prefill_matches_oracle(name, context, engine):
    # xh_prefill = the prompt loop of run_completion in one call; KV rings and the last logits
    # equal the oracle's token-by-token forward
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf, context=context)
    configure(gm, engine)
    om = O.OracleModel.from_xalm(xf, context=context)
    toks = [1] + [3 + (i * 29) % 290 for i in range(36)]
    st = InferenceState(gm.config)
    gm.prefill(toks, 0, st)
    for pos, tok in enumerate(toks):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
    # a prompt that wraps the ring takes the token loop
    check(st.logits(), om.logits(), name, "prefill" if len(toks) <= gm.config.max_seq_len else "loop")
    n = min(len(toks), gm.config.max_seq_len)
    for layer in range(gm.config.n_layers):
        a = gm.kv_read(layer, 1, 0, n).view(np.float16).astype(np.float32)
        b = om.kv(layer, 1)[:n].view(np.float16).astype(np.float32)
        assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max())


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("n", [2, 37, 64, 150])
def test_batched_prefill_matches_oracle(name, n, mode):
    """xh_prefill's batched path (prefill.h / gemm16.h: the LDS-tiled f16 MFMA GEMM over passes of
    <= PF_TOK_MM = 2048 tokens for f16 / fp8 weights, register-streaming MFMA GEMMs over passes of <= 64 tokens
    otherwise; causal attention on MFMA tiles) vs the oracle's token-by-token HYDRATE loop: last
    logits, every layer's K and V rows, and the greedy continuation after it.  mode 1: the default
    choice per dtype; 2: split-f16 register-streaming MFMA wherever the weights allow (f16 / fp8);
    3: f32-input MFMA; 4: mode 1 with hipBLASLt in place of gemm16.h."""
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf, context=256)
    assert gm.get_option(L.OPT_PREFILL) == 1
    gm.set_option(L.OPT_PREFILL, mode)
    assert gm.get_option(L.OPT_PREFILL) == mode
    om = O.OracleModel.from_xalm(xf, context=256)
    toks = [1] + [3 + (i * 37) % 280 for i in range(n - 1)]
    st = InferenceState(gm.config)
    gm.prefill(toks, 0, st)
    for pos, tok in enumerate(toks):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
    check(st.logits(), om.logits(), name, "prefill")
    for layer in range(gm.config.n_layers):
        for which in (0, 1):
            a = gm.kv_read(layer, which, 0, n).view(np.float16).astype(np.float32)
            b = om.kv(layer, which)[:n].view(np.float16).astype(np.float32)
            assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), (layer, which)
    nxt = gm.decode_greedy(n, 3)
    gm.get_logits(st)
    for i, t in enumerate(nxt):
        om.forward(t, n + i)
    check(st.logits(), om.logits(), name, "prefill")


@pytest.mark.parametrize("mode,n", [(1, 2200), (4, 700)])
@pytest.mark.parametrize("name", ["tiny_mistral_f16", "tiny_mistral_f8_e4m3", "small_llama_f16"])
def test_multi_pass_prefill_matches_oracle(name, mode, n):
    """XH_OPT_PREFILL 1 on f16 / fp8 weights: gemm16.h passes of 2048 tokens (2200 tokens = a full
    pass and a 152-token one, the second attending over the first pass's K/V rows); 4: hipBLASLt
    passes of 512 (700 = 512 + 188).  Last logits and every layer's K/V rows vs the oracle's token
    loop, then the perplexity path over 600 tokens (lm_head as one GEMM per pass, or 64-token
    slices for bf16 lm_heads)."""
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf, context=4096)
    gm.set_option(L.OPT_PREFILL, mode)
    om = O.OracleModel.from_xalm(xf, context=4096)
    toks = [1] + [3 + (i * 37) % 280 for i in range(n - 1)]
    st = InferenceState(gm.config)
    gm.prefill(toks, 0, st)
    for pos, tok in enumerate(toks):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
    check(st.logits(), om.logits(), name, "prefill")
    for layer in range(gm.config.n_layers):
        for which in (0, 1):
            a = gm.kv_read(layer, which, 0, n).view(np.float16).astype(np.float32)
            b = om.kv(layer, which)[:n].view(np.float16).astype(np.float32)
            assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), (layer, which)
    gm.close()
    gm2 = Model.from_xalm(xf, context=4096)
    gm2.set_option(L.OPT_PREFILL, mode)
    om2 = O.OracleModel.from_xalm(xf, context=4096)
    check_probs(gm2.token_probs(toks[:600]), om2, toks[:600], name)


@pytest.mark.parametrize("mode", [1, 4])
@pytest.mark.parametrize("wdt", [L.F16, L.F8_E4M3])
def test_prefill_is_deterministic_across_contexts(wdt, mode):
    """Two fresh contexts prefill the same 300-token prompt to bitwise-equal logits and K/V rows:
    the GEMMs' summation order is fixed (gemm16.h tiling; hipBLASLt: the heuristic's first
    algorithm, no run-time timing of candidates)."""
    toks = [1] + [3 + (i * 37) % 500 for i in range(299)]
    out = []
    for _ in range(2):
        gm, _om = synthetic_pair(wdt, context=512)
        gm.set_option(L.OPT_PREFILL, mode)
        st = InferenceState(gm.config)
        gm.prefill(toks, 0, st)
        out.append((st.logits().copy(), gm.kv_read(1, 0, 0, len(toks)).copy()))
        gm.close()
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32))
    assert np.array_equal(out[0][1], out[1][1])


def synthetic_pair(wdt, dim=256, hidden=512, n_layers=2, vocab=512, context=256):
    """The same synthetic weights (include/xalm_synth.h) in a device Model and the oracle."""
    cfg = L.XhConfig()
    cfg.dim, cfg.hidden_dim, cfg.head_dim, cfg.n_layers = dim, hidden, 64, n_layers
    cfg.n_heads, cfg.n_kv_heads, cfg.vocab_size, cfg.max_seq_len = 4, 1, vocab, context
    cfg.rope_theta, cfg.rotary_dim, cfg.norm_eps, cfg.act = 1e6, 64, 1e-5, L.ACT_SILU
    cfg.qkv_clip, cfg.tie_word_embeddings = float(np.finfo(np.float32).max), 0
    gm, om = Model(cfg), O.OracleModel(cfg)
    q_dim, kv_dim = cfg.n_heads * cfg.head_dim, cfg.n_kv_heads * cfg.head_dim
    shape = {L.EMBED: (vocab, dim), L.WCLS: (vocab, dim), L.FINAL_NORM: (1, dim), L.ATTN_NORM: (1, dim),
             L.FFN_NORM: (1, dim), L.WQ: (q_dim, dim), L.WK: (kv_dim, dim), L.WV: (kv_dim, dim),
             L.WO: (dim, q_dim), L.W1: (hidden, dim), L.W2: (dim, hidden), L.W3: (hidden, dim)}
    specs = [(L.EMBED, 0, L.F16, 11, 0.0, 1.0), (L.WCLS, 0, L.F16, 12, 0.0, 0.05),
             (L.FINAL_NORM, 0, L.BF16, 13, 1.0, 0.01)]
    for layer in range(n_layers):
        for i, kind in enumerate([L.WQ, L.WK, L.WV, L.WO, L.W1, L.W2, L.W3]):
            specs.append((kind, layer, wdt, 100 + 10 * layer + i, 0.0, 0.05))
        specs += [(L.ATTN_NORM, layer, L.BF16, 300 + layer, 1.0, 0.01), (L.FFN_NORM, layer, L.BF16, 400 + layer, 1.0, 0.01)]
    for kind, layer, dt, seed, mean, std in specs:
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
        rows, cols = shape[kind]
        om.set_tensor(kind, layer, dt, O.synthetic(rows, cols, dt, seed, mean, std))
    return gm, om


@pytest.mark.parametrize("glu", [1, 0])
@pytest.mark.parametrize("mode", [1, 2, 3, 4])
@pytest.mark.parametrize("wdt", [L.F16, L.F8_E4M3, L.F8_E5M2])
def test_prefill_gemm_paths_on_synthetic_weights(wdt, mode, glu):
    # dims (256 / 512) that take the split-f16 kernel for fp8 too (K % 8E); 100 tokens = a full
    # pass and a partial one; logits vs the oracle's token loop, then the perplexity path.
    # glu 0 routes the W2 input through the f32 GLU epilogue + split pass instead of the fused one
    gm, om = synthetic_pair(wdt)
    gm.set_option(L.OPT_PREFILL, mode)
    gm.set_option(L.OPT_PREFILL_GLU_SPLIT, glu)
    toks = [1] + [3 + (i * 37) % 500 for i in range(99)]
    st = InferenceState(gm.config)
    gm.prefill(toks, 0, st)
    for pos, tok in enumerate(toks):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
    ref = om.logits()
    assert np.isfinite(st.logits()).all()
    check(st.logits(), ref)
    gm2, om2 = synthetic_pair(wdt)
    gm2.set_option(L.OPT_PREFILL, mode)
    gm2.set_option(L.OPT_PREFILL_GLU_SPLIT, glu)
    check_probs(gm2.token_probs(toks[:70]), om2, toks[:70])


@pytest.mark.parametrize("wdt", [L.F16, L.BF16, L.F8_E4M3, L.F8_E5M2])
def test_pipelined_gemv_decode(wdt):
    # dim 4096: the qkv and W1/W3 launches take the pipelined gemv shape (gemv_rows_pipe, n a
    # multiple of 64 E U: 2048 for 2-byte weights, 4096 for fp8) with 3 (W1/W3) and 1 (qkv) row
    # groups per wave; token-loop logits at every position and the device greedy loop vs the oracle
    gm, om = synthetic_pair(wdt, dim=4096, hidden=2048, n_layers=1)
    st = InferenceState(gm.config)
    toks = [1, 17, 300, 5, 99, 250]
    for pos, tok in enumerate(toks):
        gm.forward(st, tok, pos, L.OUTPUT_LOGITS)
        om.forward(tok, pos)
        check(st.logits(), om.logits(), what=pos)
    nxt = gm.decode_greedy(len(toks), 3)
    gm.get_logits(st)
    for i, t in enumerate(nxt):
        om.forward(t, len(toks) + i)
    check(st.logits(), om.logits())


@pytest.mark.parametrize("wdt", [L.F8_E4M3, L.F8_E5M2, L.F16])
def test_long_row_w2_decode(wdt):
    # hidden 7168: W2 rows of 7 KiB (one-byte weights) / 14 KiB (f16) through the PF shape that
    # holds x in 8 float4 per thread, partial last step (fp8: 7 chunks per row, steps of 4);
    # token-loop logits vs the oracle at every position
    gm, om = synthetic_pair(wdt, dim=256, hidden=7168, n_layers=1)
    st = InferenceState(gm.config)
    for pos, tok in enumerate([1, 17, 300, 5]):
        gm.forward(st, tok, pos, L.OUTPUT_LOGITS)
        om.forward(tok, pos)
        check(st.logits(), om.logits(), what=pos)


@pytest.mark.parametrize("wdt", [L.F16, L.F8_E4M3])
def test_fused_glu_split_is_bit_identical(wdt):
    # the fused GLU -> split-f16 epilogue and the two-launch route produce the same W2 input
    toks = [1] + [3 + (i * 41) % 500 for i in range(99)]
    out = []
    for glu in (1, 0):
        gm, _ = synthetic_pair(wdt)
        gm.set_option(L.OPT_PREFILL, 2)
        gm.set_option(L.OPT_PREFILL_GLU_SPLIT, glu)
        assert gm.get_option(L.OPT_PREFILL_GLU_SPLIT) == glu
        st = InferenceState(gm.config)
        gm.prefill(toks, 0, st)
        out.append(st.logits().copy())
    assert np.array_equal(out[0], out[1]), float(np.abs(out[0] - out[1]).max())


@pytest.mark.parametrize("batched", [1, 2, 3, 4])
def test_batched_prefill_equals_token_loop(batched):
    """Batched and per-token prefill of the same prompt agree (logits and K/V rings)."""
    xf = XalmFile(fixture_path("small_llama_f16.xalm"))
    toks = [1] + [3 + (i * 53) % 300 for i in range(99)]
    out = []
    for mode in (batched, 0):
        gm = Model.from_xalm(xf, context=512)
        gm.set_option(L.OPT_PREFILL, mode)
        st = InferenceState(gm.config)
        gm.prefill(toks, 0, st)
        out.append((st.logits().copy(), gm.kv_read(1, 0, 0, len(toks)).view(np.float16).astype(np.float32)))
        gm.close()
    check(out[0][0], out[1][0], "small_llama_f16", "prefill")
    assert np.abs(out[0][1] - out[1][1]).max() <= 2e-3 * max(1.0, np.abs(out[1][1]).max())


def test_engines_agree_on_long_decode():
    # 120 greedy tokens on the head_dim-128 fixture: both launch structures give the same tokens
    # (same per-row math) and logits within the tolerance
    xf = XalmFile(fixture_path("small_llama_f16.xalm"))
    res = []
    for engine in ENGINES:
        gm = Model.from_xalm(xf)
        configure(gm, engine)
        st = InferenceState(gm.config)
        gm.prefill([1, 7, 99], 0, st)
        toks = gm.decode_greedy(3, 120)
        gm.get_logits(st)
        res.append((toks, st.logits().copy()))
        gm.close()
    for toks, lg in res[1:]:
        assert toks == res[0][0]
        check(lg, res[0][1], "small_llama_f16", "loop")


def test_graphs_and_eager_bitwise_equal():
    xf = XalmFile(fixture_path("small_llama_f16.xalm"))
    outs = []
    for graphs in (True, False):
        gm = Model.from_xalm(xf)
        gm.set_graphs(graphs)
        st = InferenceState(gm.config)
        for pos, tok in enumerate([1, 5, 77, 200, 9]):
            gm.forward(st, tok, pos)
        outs.append(st.logits().copy())
        gm.close()
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("engine", ENGINES)
def test_device_greedy_decode_matches_oracle_teacher_forced(engine):
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    gm = Model.from_xalm(xf)
    configure(gm, engine)
    om = O.OracleModel.from_xalm(xf)
    st = InferenceState(gm.config)
    prompt = [1, 84, 262, 259, 90]
    for pos, tok in enumerate(prompt):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
    toks = gm.decode_greedy(len(prompt), 20)
    assert len(toks) == 20
    pos = len(prompt)
    for t in toks:
        lg = om.logits()
        top2 = np.sort(lg)[-2:]
        if top2[1] - top2[0] > 1e-3:  # not a near-tie: argmax must agree exactly
            assert t == O.sample_argmax(lg)
        om.forward(t, pos)
        pos += 1
    gm.get_logits(st)
    check(st.logits(), om.logits(), "tiny_mistral_f16", "loop")


@pytest.mark.parametrize("engine", ENGINES)
def test_decode_stops_on_eos(engine):
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    gm = Model.from_xalm(xf)
    configure(gm, engine)
    st = InferenceState(gm.config)
    gm.forward(st, 1, 0)
    first = gm.decode_greedy(1, 3)
    gm.reset()
    gm.forward(st, 1, 0)
    got = gm.decode_greedy(1, 10, stop=(first[1], -1))
    assert got == first[:2]


def test_upload_validation():
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    gm = Model(xf.config())
    with pytest.raises(L.XhError):
        gm.upload(L.WQ, 0, L.F16, np.zeros(10, np.uint16))  # wrong size
    with pytest.raises(L.XhError):
        gm.upload(L.ATTN_NORM, 0, L.F16, np.zeros(64, np.uint16))  # norms are F32/BF16
    with pytest.raises(L.XhError):
        gm.upload(L.WQ, 5, L.F16, np.zeros(64 * 64, np.uint16))  # layer out of range
    st = InferenceState(gm.config)
    with pytest.raises(L.XhError):
        gm.forward(st, 1, 0)  # weights missing


def check_probs(got, om, toks, fixture=None):
    """got[i] vs the oracle's Sampler::sample_prob(toks[i+1]) after forwarding toks[i] (the
    run_perplexity loop, src/main.cpp:243-254).  Bar on |log p - log p_ref|: 2 x the logits bar
    of that position (log p moves by at most twice the worst logit error; path "ppl" of the
    fixture's envelope); probabilities the reference underflows to 0 (|logits| ~ 90 on
    small_llama) must be below 1e-30 here."""
    assert got.shape == (len(toks) - 1,)
    for pos in range(len(toks) - 1):
        om.forward(toks[pos], pos)
        lg = om.logits()
        ref = O.sample_prob(lg, toks[pos + 1])
        if ref < 1e-30:
            assert got[pos] < 1e-30, (pos, got[pos], ref)
            continue
        assert got[pos] > 0, (pos, got[pos], ref)
        check_logp(float(abs(np.log(got[pos]) - np.log(ref))), lg, fixture, pos)


@pytest.mark.parametrize("prefill", [1, 2, 3, 4, 0])
@pytest.mark.parametrize("name", ["tiny_mistral_f16", "tiny_mistral_bf16", "tiny_mistral_f8_e4m3",
                                  "small_llama_f16"])
def test_perplexity_probs_match_oracle(name, prefill):
    # xh_perplexity: batched passes (prefill 2 / 3 and bf16: 89 tokens = a full 64-token pass + 25;
    # prefill 1 / 4 on f16 / fp8: one gemm16.h / hipBLASLt pass; lm_head as one GEMM per pass) and
    # the token loop (prefill 0)
    xf = XalmFile(fixture_path(name + ".xalm"))
    gm = Model.from_xalm(xf, context=256)
    gm.set_option(L.OPT_PREFILL, prefill)
    om = O.OracleModel.from_xalm(xf, context=256)
    toks = [1] + [3 + (i * 41) % 280 for i in range(89)]
    check_probs(gm.token_probs(toks), om, toks, name)


def test_perplexity_token_loop_ring():
    # a sequence longer than -T (ring wrap + sinks): the token loop
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    ctxlen = 16
    gm = Model.from_xalm(xf, context=ctxlen)
    om = O.OracleModel.from_xalm(xf, context=ctxlen)
    toks = [1] + [3 + (i * 23) % 290 for i in range(40)]
    check_probs(gm.token_probs(toks), om, toks, "tiny_mistral_f16")


def test_prefill_option_values():
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    gm = Model.from_xalm(xf)
    assert gm.get_option(L.OPT_PREFILL) == 1
    for v in (0, 2, 3, 4, 1):
        gm.set_option(L.OPT_PREFILL, v)
        assert gm.get_option(L.OPT_PREFILL) == v
    for bad in (-1, 5):
        with pytest.raises(L.XhError):
            gm.set_option(L.OPT_PREFILL, bad)
    assert gm.get_option(L.OPT_PREFILL) == 1
    # option id 4 (the removed XH_OPT_COL_KV_MAX) is rejected, not reinterpreted
    with pytest.raises(L.XhError):
        gm.set_option(4, 0)
    with pytest.raises(L.XhError):
        gm.get_option(4)
    assert L.OPT_PREFILL_ATTN == 5 and gm.get_option(L.OPT_PREFILL_ATTN) == 1


def test_perplexity_arguments():
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    gm = Model.from_xalm(xf)
    with pytest.raises(L.XhError):
        gm.token_probs([1])  # needs a target
    with pytest.raises(L.XhError):
        gm.token_probs([1, 10 ** 6])  # target out of range


@pytest.mark.parametrize("name", FIXTURES)
def test_upload_file_equals_host_upload(name):
    # xh_upload_file (pread into pinned staging + DMA) and xh_upload (host buffer) must leave
    # the same bytes on the device: the logits agree bit for bit
    xf = XalmFile(fixture_path(name + ".xalm"))
    outs = []
    for direct in (True, False):
        gm = Model.from_xalm(xf, direct=direct)
        st = InferenceState(gm.config)
        got = []
        for pos, tok in enumerate([1, 5, 9, 3]):
            gm.forward(st, tok, pos)
            got.append(st.logits().copy())
        outs.append(np.stack(got))
        gm.close()
    assert np.array_equal(outs[0], outs[1])


def test_upload_file_multi_chunk_strided(tmp_path):
    # Mistral-7B gate/up shapes (f16 [14336, 4096] = 112 MiB each, at a nonzero file offset)
    # into the interleaved W1/W3 slot: file upload vs host upload, bit-equal logits
    cfg = L.XhConfig()
    cfg.dim, cfg.hidden_dim, cfg.head_dim, cfg.n_layers = 4096, 14336, 128, 1
    cfg.n_heads, cfg.n_kv_heads, cfg.vocab_size, cfg.max_seq_len = 32, 8, 512, 64
    cfg.rope_theta, cfg.rotary_dim, cfg.norm_eps, cfg.act = 1e6, 128, 1e-5, L.ACT_SILU
    cfg.qkv_clip, cfg.tie_word_embeddings = float(np.finfo(np.float32).max), 0
    rng = np.random.default_rng(3)
    w = {k: (rng.standard_normal((14336, 4096), dtype=np.float32) * 0.02).astype(np.float16).view(np.uint16)
         for k in (L.W1, L.W3)}
    path = tmp_path / "w13.bin"
    with open(path, "wb") as f:
        f.write(b"\0" * 96)  # a nonzero, 32-B aligned start, as in a .xalm file
        for k in (L.W1, L.W3):
            f.write(w[k].tobytes())
    outs = []
    for direct in (True, False):
        gm = Model(cfg)
        for i, kind in enumerate([L.EMBED, L.WQ, L.WK, L.WV, L.WO, L.W2, L.WCLS]):
            gm.upload_synthetic(kind, 0, L.F16, 100 + i, 0.0, 1.0 if kind == L.EMBED else 0.02)
        for kind in (L.ATTN_NORM, L.FFN_NORM, L.FINAL_NORM):
            gm.upload_synthetic(kind, 0, L.BF16, 200 + kind, 1.0, 0.01)
        for j, kind in enumerate((L.W1, L.W3)):
            if direct:
                gm.upload_file(kind, 0, L.F16, str(path), 96 + j * w[kind].nbytes, w[kind].nbytes)
            else:
                gm.upload(kind, 0, L.F16, w[kind])
        st = InferenceState(cfg)
        gm.forward(st, 7, 0)
        outs.append(st.logits().copy())
        gm.close()
    assert np.isfinite(outs[0]).all()
    assert np.array_equal(outs[0], outs[1])


def test_upload_file_validation(tmp_path):
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    gm = Model(xf.config())
    ti = xf.tensors["l.0.attn.q.weight"]
    with pytest.raises(L.XhError):
        gm.upload_file(L.WQ, 0, L.F16, str(tmp_path / "missing.xalm"), ti.offset, ti.size)
    with pytest.raises(L.XhError):  # range past the end of the file
        gm.upload_file(L.WQ, 0, L.F16, xf.path, ti.offset + 10 ** 9, ti.size)
    with pytest.raises(L.XhError):  # wrong size
        gm.upload_file(L.WQ, 0, L.F16, xf.path, ti.offset, ti.size - 2)
    short = tmp_path / "short.bin"
    short.write_bytes(b"\0" * 100)
    with pytest.raises(L.XhError):
        gm.upload_file(L.WQ, 0, L.F16, str(short), 0, ti.size)
    gm.upload_file(L.WQ, 0, L.F16, xf.path, ti.offset, ti.size)  # the good call still works


@pytest.mark.parametrize("engine", ENGINES)
def test_multi_split_attention_in_model(engine):
    # -T 1024 on the head_dim-128 fixture: kv_len 300 runs attention in several splits whose
    # partials are merged in-launch (ticket), inside the fused attention + Wo launch too
    xf = XalmFile(fixture_path("small_llama_f16.xalm"))
    gm = Model.from_xalm(xf, context=1024)
    configure(gm, engine)
    om = O.OracleModel.from_xalm(xf, context=1024)
    toks = [1] + [3 + (i * 71) % 310 for i in range(299)]
    st = InferenceState(gm.config)
    gm.prefill(toks, 0, st)
    for pos, tok in enumerate(toks):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
    check(st.logits(), om.logits(), "small_llama_f16", "prefill")
    nxt = gm.decode_greedy(len(toks), 4)
    assert len(nxt) == 4
    gm.get_logits(st)
    for i, t in enumerate(nxt):
        om.forward(t, len(toks) + i)
    check(st.logits(), om.logits(), "small_llama_f16", "prefill")


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("history", [20000, 32767])
def test_long_context_streaming_attention(engine, history):
    """Synthetic GQA model (8 KV heads x head_dim 128, 4 q per KV, -T 32768) with a filled KV
    history: splits longer than one prefetch round take the streaming online-softmax form
    (attention.h attn_block_stream) inside the fused attention + Wo launch.  One forward at
    pos = history vs the oracle on the same weights and the same KV rows."""
    import bench

    w = dict(dim=512, hidden=512, layers=2, heads=32, kv_heads=8, head_dim=128, vocab=256, msl=32768, theta=1e6,
             wdt=L.F16, edt=L.F16, cdt=L.F16)
    c = bench.make_config(w)
    gm = Model(c)
    configure(gm, engine)
    om = O.OracleModel(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
        rows, cols = bench.tensor_shape(c, kind)
        om.set_tensor(kind, layer, dt, O.synthetic(rows, cols, dt, seed, mean, std))
    kv_dim = c.n_kv_heads * c.head_dim
    for layer in range(c.n_layers):
        for which in (0, 1):
            seed = 700 + 2 * layer + which
            gm.kv_fill_synthetic(layer, which, 0, history, seed, 1.0)
            om.set_kv(layer, which, 0, O.synthetic(history, kv_dim, L.F16, seed, 0.0, 1.0))
    st = InferenceState(c)
    gm.forward(st, 17, history, L.OUTPUT_LOGITS)
    om.forward(17, history, L.OUTPUT_LOGITS)
    check(st.logits(), om.logits())
    gm.close()
    om.close()
