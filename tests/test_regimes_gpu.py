"""Parity in the regimes the fixture tests do not reach (VERDICT r2 "What's missing" 1-4).

* configs[3]'s timed path: the device greedy loop (xh_decode_greedy: argmax_embed_kernel
  advances StepParams with step_positions) across the ring wrap at -T 32768 with the StreamingLLM
  sinks active (src/infer.cpp:608-613 kv_sink / kv_pos / kv_len; :416-431 sink re-rotation), and
  the same at -T 16 on the converter fixture;
* a Llama-3-sized lm_head (V = 128256, dim 4096) and the device argmax over its workgroup
  candidates against Sampler::sample_argmax (src/sampler.cpp:19-30: FLT_MIN start, first max);
* a finite qkv_clip (src/infer.cpp:392-399, src/model.h:84-85) and the GELU activation
  (src/infer.cpp:299-301, :472-477), every other test runs FLT_MAX / SiLU;
* xh_active_bytes (the roofline numerator) against Model::active_bytes (src/model.cpp:12-35),
  restated here in Python and in the oracle, for every dtype, tied and untied lm_head.
"""
import numpy as np
import pytest

from conftest import fixture_path
from oracle import oracle as O
from xalm_amd import _lib as L
from xalm_amd.model import InferenceState, Model
from xalm_amd.xalm_file import XalmFile

pytestmark = pytest.mark.gpu

FLT_MAX = float(np.finfo(np.float32).max)


def make_cfg(dim, hidden, layers, heads, kv_heads, head_dim, vocab, msl, theta=1e6, act=L.ACT_SILU,
             qkv_clip=FLT_MAX, tied=0):
    c = L.XhConfig()
    c.dim, c.hidden_dim, c.head_dim, c.n_layers = dim, hidden, head_dim, layers
    c.n_heads, c.n_kv_heads, c.vocab_size, c.max_seq_len = heads, kv_heads, vocab, msl
    c.rope_theta, c.rotary_dim, c.norm_eps, c.act = theta, head_dim, 1e-5, act
    c.qkv_clip, c.tie_word_embeddings = qkv_clip, tied
    return c


def shapes(c):
    q_dim, kv_dim = c.n_heads * c.head_dim, c.n_kv_heads * c.head_dim
    return {L.EMBED: (c.vocab_size, c.dim), L.WCLS: (c.vocab_size, c.dim), L.FINAL_NORM: (1, c.dim),
            L.ATTN_NORM: (1, c.dim), L.FFN_NORM: (1, c.dim), L.WQ: (q_dim, c.dim), L.WK: (kv_dim, c.dim),
            L.WV: (kv_dim, c.dim), L.WO: (c.dim, q_dim), L.W1: (c.hidden_dim, c.dim),
            L.W2: (c.dim, c.hidden_dim), L.W3: (c.hidden_dim, c.dim)}


def build_pair(c, wdt, edt=None, cdt=None, wstd=0.05, cstd=0.05):
    """Device Model and oracle on the same synthetic weights (include/xalm_synth.h)."""
    edt = wdt if edt is None else edt
    cdt = edt if cdt is None else cdt
    gm, om = Model(c), O.OracleModel(c)
    sh = shapes(c)
    specs = [(L.EMBED, 0, edt, 11, 0.0, 1.0), (L.FINAL_NORM, 0, L.BF16, 13, 1.0, 0.01)]
    if not c.tie_word_embeddings:
        specs.append((L.WCLS, 0, cdt, 12, 0.0, cstd))
    for layer in range(c.n_layers):
        for i, kind in enumerate([L.WQ, L.WK, L.WV, L.WO, L.W1, L.W2, L.W3]):
            specs.append((kind, layer, wdt, 100 + 10 * layer + i, 0.0, wstd))
        specs += [(L.ATTN_NORM, layer, L.BF16, 300 + layer, 1.0, 0.01),
                  (L.FFN_NORM, layer, L.BF16, 400 + layer, 1.0, 0.01)]
    for kind, layer, dt, seed, mean, std in specs:
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
        rows, cols = sh[kind]
        arr = O.synthetic(rows, cols, dt, seed, mean, std)
        om.set_tensor(kind, layer, dt, arr)
        if kind == L.EMBED and c.tie_word_embeddings:
            om.set_tensor(L.WCLS, 0, dt, arr)  # Model::from_xalm loads embed.weight as wcls
    return gm, om


def bar(ref):
    # the north-star bar: 1e-3 max-abs, stated relative to the logit scale above 1
    return 1e-3 * max(1.0, float(np.abs(ref).max()))


def f16(a):
    return a.view(np.float16).astype(np.float32)


def check_teacher_forced(gm, om, toks, pos0, st):
    """The device greedy tokens vs Sampler::sample_argmax of the oracle fed the same tokens;
    a near-tie (top-2 margin within the logits bar) may go either way.  Returns the number of
    exact agreements."""
    agree = 0
    for i, t in enumerate(toks):
        lg = om.logits()
        top2 = np.sort(lg)[-2:]
        if top2[1] - top2[0] > 2 * bar(lg):
            assert t == O.sample_argmax(lg), (i, t, O.sample_argmax(lg), float(top2[1] - top2[0]))
        agree += int(t == O.sample_argmax(lg))
        om.forward(t, pos0 + i)
    gm.get_logits(st)
    assert np.abs(st.logits() - om.logits()).max() <= bar(om.logits())
    return agree


# ---------------------------------------------------------------------------------------------
# (a) the ring wrap with sinks on the device decode loop
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("fuse", [1, 0])
def test_decode_greedy_across_wrap_32k(fuse):
    """configs[3]: 8 KV heads x head_dim 128, 4 q per KV, -T 32768.  Slots 0..32766 hold a
    synthetic history; forward the token at pos 32767 (ring full, no sinks yet), then 4 greedy
    steps on the device at pos 32768..32771: kv_sink = 2, kv_pos = 2 + (pos - 2) % 32766 (the
    ring wraps onto slots 2..5), both sink K rows re-rotated by rope(pos = 1) every step.
    Logits, argmax, sink K rows and the overwritten ring rows vs the teacher-forced oracle."""
    msl, hist = 32768, 32767
    c = make_cfg(512, 512, 2, 32, 8, 128, 256, msl)
    gm, om = build_pair(c, L.F16, wstd=0.02)
    gm.set_option(L.OPT_FUSE_ATTN_WO, fuse)
    kv_dim = c.n_kv_heads * c.head_dim
    for layer in range(c.n_layers):
        for which in (0, 1):
            seed = 900 + 2 * layer + which
            gm.kv_fill_synthetic(layer, which, 0, hist, seed, 1.0)
            om.set_kv(layer, which, 0, O.synthetic(hist, kv_dim, L.F16, seed, 0.0, 1.0))
    st = InferenceState(c)
    gm.forward(st, 17, hist)
    om.forward(17, hist)
    assert np.abs(st.logits() - om.logits()).max() <= bar(om.logits())
    toks = gm.decode_greedy(hist + 1, 4)
    assert len(toks) == 4
    check_teacher_forced(gm, om, toks, hist + 1, st)
    for layer in range(c.n_layers):
        # sink K rows: rotated 4 times (f32 rope at pos 1, fp16 round trip each time); the
        # device uses host-libm cos/sin as the oracle, so they agree to one fp16 ulp
        a, b = f16(gm.kv_read(layer, 0, 0, 2)), f16(om.kv(layer, 0)[:2])
        assert np.all(np.abs(a - b) <= np.abs(b) * 2.0 ** -10 + 2.0 ** -24), (layer, float(np.abs(a - b).max()))
        # the history the sinks started from is gone: the rows did rotate
        assert not np.array_equal(a, f16(O.synthetic(hist, kv_dim, L.F16, 900 + 2 * layer, 0.0, 1.0)[:2]))
        for which in (0, 1):  # wrapped slots 2..5 hold the 4 decoded tokens' K / V
            a, b = f16(gm.kv_read(layer, which, 2, 4)), f16(om.kv(layer, which)[2:6])
            assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), (layer, which)
        # slot 6 onwards still holds the synthetic history
        a = gm.kv_read(layer, 1, 6, 4)
        assert np.array_equal(a, om.kv(layer, 1)[6:10])
    gm.close()
    om.close()


@pytest.mark.parametrize("fuse", [1, 0])
def test_decode_greedy_across_wrap_fixture(fuse):
    """-T 16 on the converter-written tiny_mistral: 6 prompt tokens, then 30 device greedy steps
    crossing pos 16 (sinks on from the wrap on, the ring lapping twice)."""
    xf = XalmFile(fixture_path("tiny_mistral_f16.xalm"))
    gm = Model.from_xalm(xf, context=16)
    gm.set_option(L.OPT_FUSE_ATTN_WO, fuse)
    om = O.OracleModel.from_xalm(xf, context=16)
    st = InferenceState(gm.config)
    prompt = [1, 84, 262, 259, 90, 282]
    for pos, tok in enumerate(prompt):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
    toks = gm.decode_greedy(len(prompt), 30)
    assert len(toks) == 30
    check_teacher_forced(gm, om, toks, len(prompt), st)
    for layer in range(gm.config.n_layers):
        a, b = f16(gm.kv_read(layer, 0, 0, 16)), f16(om.kv(layer, 0)[:16])
        assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), layer


# ---------------------------------------------------------------------------------------------
# (b) a Llama-3 vocabulary lm_head and the device argmax
# ---------------------------------------------------------------------------------------------
def test_llama3_vocab_lm_head_and_argmax():
    """V = 128256, dim 4096, Llama-3 head layout, one layer: logits at every prompt position vs
    the oracle, then 8 device greedy steps vs Sampler::sample_argmax teacher-forced (exact
    wherever the top-2 margin exceeds twice the logits bar)."""
    c = make_cfg(4096, 1024, 1, 32, 8, 128, 128256, 256, theta=5e5)
    gm, om = build_pair(c, L.F16, edt=L.F16, wstd=0.02, cstd=0.02)
    st = InferenceState(c)
    prompt = [128000, 791, 4062, 14198, 39935, 35308]
    margins = []
    for pos, tok in enumerate(prompt):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        ref = om.logits()
        assert np.abs(st.logits() - ref).max() <= bar(ref), pos
        top2 = np.sort(ref)[-2:]
        margins.append(float(top2[1] - top2[0]))
    toks = gm.decode_greedy(len(prompt), 8)
    assert len(toks) == 8
    agree = check_teacher_forced(gm, om, toks, len(prompt), st)
    assert agree >= 6, (agree, margins)
    gm.close()
    om.close()


def test_argmax_first_index_and_flt_min_quirks():
    """sample_argmax's two quirks through the device candidates (argmax_embed_kernel): the FIRST
    index of a repeated maximum wins, and logits that are all <= FLT_MIN give token 0.  Tied
    embedding with rows 5 and 9 equal and 10x the others: token 5's hidden state is dominated by
    that row, so logits 5 and 9 are the equal maxima.  A zero final norm makes every logit 0."""
    c = make_cfg(256, 512, 1, 4, 1, 64, 512, 64, tied=1)
    gm, om = build_pair(c, L.F16)
    emb = O.synthetic(512, 256, L.F16, 11, 0.0, 1.0)
    big = (emb[5].view(np.float16).astype(np.float32) * 10).astype(np.float16).view(np.uint16)
    emb[5] = big
    emb[9] = big
    gm.upload(L.EMBED, 0, L.F16, emb)
    om.set_tensor(L.EMBED, 0, L.F16, emb)
    om.set_tensor(L.WCLS, 0, L.F16, emb)
    st = InferenceState(c)
    gm.forward(st, 5, 0)
    om.forward(5, 0)
    ref = om.logits()
    assert ref[5] == ref[9] == ref.max()
    assert st.logits()[5] == st.logits()[9]
    assert gm.decode_greedy(1, 1) == [5] and O.sample_argmax(ref) == 5
    zero = np.zeros(256, np.float32)
    gm.upload(L.FINAL_NORM, 0, L.F32, zero)
    om.set_tensor(L.FINAL_NORM, 0, L.F32, zero)
    gm.reset()
    om.reset()
    gm.forward(st, 5, 0)
    om.forward(5, 0)
    assert not st.logits().any() and not om.logits().any()
    assert gm.decode_greedy(1, 1) == [0] and O.sample_argmax(om.logits()) == 0
    gm.close()
    om.close()


# ---------------------------------------------------------------------------------------------
# (c) finite qkv_clip and GELU
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("act,clip", [(L.ACT_SILU, 0.5), (L.ACT_GELU, FLT_MAX), (L.ACT_GELU, 0.5)])
def test_qkv_clip_and_gelu(act, clip):
    """qkv_clip = 0.5 clamps most q/k/v values (std ~0.8 here), GELU replaces SiLU in the GLU:
    the token loop, the device greedy loop and the batched prompt path vs the oracle."""
    c = make_cfg(256, 512, 2, 4, 1, 64, 512, 256, act=act, qkv_clip=clip)
    gm, om = build_pair(c, L.F16)
    st = InferenceState(c)
    toks = [1, 17, 300, 5, 99, 250, 7, 8]
    for pos, tok in enumerate(toks):
        gm.forward(st, tok, pos)
        om.forward(tok, pos)
        assert np.abs(st.logits() - om.logits()).max() <= bar(om.logits()), pos
    nxt = gm.decode_greedy(len(toks), 6)
    check_teacher_forced(gm, om, nxt, len(toks), st)
    # the K ring holds clipped values: every |k| <= clip before rope (rope preserves pair norms)
    if clip < FLT_MAX:
        v = f16(gm.kv_read(0, 1, 0, len(toks)))
        assert np.abs(v).max() <= clip * (1 + 2 ** -10)
    # batched prompt path (prefill.h epilogues: clip + GELU)
    for mode in (1, 2, 3):
        gm2, om2 = build_pair(c, L.F16)
        gm2.set_option(L.OPT_PREFILL, mode)
        p = [1] + [3 + (i * 37) % 500 for i in range(69)]
        gm2.prefill(p, 0, st)
        for pos, tok in enumerate(p):
            om2.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(p) - 1 else L.HYDRATE_KV_CACHE)
        assert np.abs(st.logits() - om2.logits()).max() <= bar(om2.logits()), mode
        gm2.close()
        om2.close()


# ---------------------------------------------------------------------------------------------
# (d) xh_active_bytes == Model::active_bytes
# ---------------------------------------------------------------------------------------------
BITS = {L.F32: 32, L.F16: 16, L.BF16: 16, L.F8_E4M3: 8, L.F8_E5M2: 8, L.Q8: 8}


def ref_active_bytes(c, dts, pos):
    """src/model.cpp:12-35 restated: type.bit_size / 8 per element (gguf blocks, which the C++
    runtime cannot parse, at their block bytes: 34 / 18 per 32 elements)."""
    def nbytes(dt, n):
        return n // 32 * L.GQ_BLOCK_BYTES[dt] if dt in L.GQ_BLOCK_BYTES else n * BITS[dt] // 8
    q_dim, kv_dim = c.n_heads * c.head_dim, c.n_kv_heads * c.head_dim
    b = nbytes(dts["embed"], c.dim) + nbytes(L.BF16, c.dim) + c.vocab_size * nbytes(dts["wcls"], c.dim)
    for _ in range(c.n_layers):
        b += 2 * nbytes(L.BF16, c.dim)
        b += q_dim * nbytes(dts["w"], c.dim) + 2 * kv_dim * nbytes(dts["w"], c.dim)
        b += c.dim * nbytes(dts["w"], q_dim)
        b += 2 * c.hidden_dim * nbytes(dts["w"], c.dim) + c.dim * nbytes(dts["w"], c.hidden_dim)
        b += 2 * min(c.max_seq_len, pos + 1) * kv_dim * 2
    return b


@pytest.mark.parametrize("tied", [0, 1])
@pytest.mark.parametrize("wdt,edt", [(L.F32, L.F32), (L.F16, L.F16), (L.BF16, L.BF16), (L.F8_E4M3, L.BF16),
                                     (L.F8_E5M2, L.BF16), (L.F8_E4M3, L.F8_E4M3), (L.Q8_0, L.Q8_0),
                                     (L.Q4_0, L.Q4_0), (L.F16, L.Q8_0)])
def test_active_bytes_matches_reference_formula(wdt, edt, tied):
    c = make_cfg(256, 512, 2, 4, 2, 64, 512, 128, tied=tied)
    gm, om = build_pair(c, wdt, edt=edt)
    dts = {"w": wdt, "embed": edt, "wcls": edt}
    for pos in (0, 1, 100, 127, 128, 1000):
        ref = ref_active_bytes(c, dts, pos)
        assert gm.active_bytes(pos) == ref, (pos, gm.active_bytes(pos), ref)
        assert om.active_bytes(pos) == ref, (pos, om.active_bytes(pos), ref)
    gm.close()
    om.close()


def test_active_bytes_q8_matrices():
    # Type::Q8 (int8 x 0.01, src/types.h:423-424) has no synthetic fill: host upload
    c = make_cfg(256, 512, 1, 4, 2, 64, 512, 128)
    gm = Model(c)
    sh = shapes(c)
    rng = np.random.default_rng(1)
    for kind in (L.WQ, L.WK, L.WV, L.WO, L.W1, L.W2, L.W3):
        gm.upload(kind, 0, L.Q8, rng.integers(-100, 100, sh[kind], dtype=np.int8))
    for kind, dt in ((L.EMBED, L.F16), (L.WCLS, L.F16)):
        gm.upload_synthetic(kind, 0, dt, 5, 0.0, 1.0)
    for kind in (L.ATTN_NORM, L.FFN_NORM, L.FINAL_NORM):
        gm.upload_synthetic(kind, 0, L.BF16, 6, 1.0, 0.01)
    dts = {"w": L.Q8, "embed": L.F16, "wcls": L.F16}
    for pos in (0, 50, 500):
        assert gm.active_bytes(pos) == ref_active_bytes(c, dts, pos)
    gm.close()


# ---------------------------------------------------------------------------------------------
# Mistral-width layers: both launch structures, with and without a KV history
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("history", [0, 300, 3000])
@pytest.mark.parametrize("wdt", [L.F16, L.BF16, L.F8_E4M3, L.F8_E5M2])
@pytest.mark.parametrize("fuse", [1, 0])
def test_launch_structures_match_oracle(wdt, history, fuse):
    """dim 4096 with 32 q heads x 128 (the fused attention + Wo launch holds the Wo rows in
    registers across the hand-off): attention + Wo in one launch (1) or two (0), against the
    oracle, token loop and device greedy loop; `history` slots of synthetic K/V first (several
    attention splits; merged partials at 3000)."""
    c = make_cfg(4096, 2048, 2, 32, 8, 128, 512, 4096)
    kv_dim = c.n_kv_heads * c.head_dim
    gm, om = build_pair(c, wdt, edt=L.BF16 if wdt in (L.F8_E4M3, L.F8_E5M2) else wdt, wstd=0.02)
    gm.set_option(L.OPT_FUSE_ATTN_WO, fuse)
    assert gm.get_option(L.OPT_FUSE_ATTN_WO) == fuse
    for layer in range(c.n_layers):
        for which in (0, 1):
            if history:
                seed = 1200 + 2 * layer + which
                gm.kv_fill_synthetic(layer, which, 0, history, seed, 1.0)
                om.set_kv(layer, which, 0, O.synthetic(history, kv_dim, L.F16, seed, 0.0, 1.0))
    st = InferenceState(c)
    toks = [1, 17, 300, 5]
    for i, tok in enumerate(toks):
        gm.forward(st, tok, history + i)
        om.forward(tok, history + i)
        assert np.abs(st.logits() - om.logits()).max() <= bar(om.logits()), i
    nxt = gm.decode_greedy(history + len(toks), 6)
    check_teacher_forced(gm, om, nxt, history + len(toks), st)
    # the hand-off words were left clean for the next step (check_aw reports a timeout)
    gm.forward(st, 3, history + len(toks) + 6)
    gm.close()
    om.close()


# (full Mistral-7B / fp8 / Llama-3 / 32k size parity against the fp64 evaluation of the reference
# algorithm: tests/test_parity_full_gpu.py)


@pytest.mark.parametrize("attn", [1, 2, 0])
@pytest.mark.parametrize("heads,kv_heads,head_dim,wdt", [(8, 2, 128, L.F16), (16, 2, 128, L.F16),
                                                          (8, 8, 128, L.F16), (8, 4, 128, L.F16), (16, 2, 64, L.F16),
                                                          (8, 2, 64, L.F8_E4M3), (4, 2, 16, L.BF16)])
def test_prompt_attention_in_two_prompts(heads, kv_heads, head_dim, wdt, attn):
    """xh_prefill's causal attention (XH_OPT_PREFILL_ATTN 1: MFMA tiles shared by a workgroup's
    waves; 2: per-wave MFMA tiles; 0: per-token split kernel) at the instantiated head shapes (QPK
    1 / 2 / 4 / 8 — MHA through GQA —, head_dim 128 / 64 / 16), a prompt
    of 600 tokens followed by a second prompt of 300 at pos 600 (its rows attend over the first
    prompt's K/V), against the oracle's token loop: last logits and every K/V row.  f16
    weights run 512-token passes (attention over a pass boundary), bf16 64-token ones."""
    c = make_cfg(256, 512, 2, heads, kv_heads, head_dim, 512, 1024)
    gm, om = build_pair(c, wdt)
    gm.set_option(L.OPT_PREFILL_ATTN, attn)
    assert gm.get_option(L.OPT_PREFILL_ATTN) == attn
    toks = [1] + [3 + (i * 37) % 500 for i in range(899)]
    st = InferenceState(c)
    gm.prefill(toks[:600], 0, st)
    gm.prefill(toks[600:], 600, st)
    for pos, tok in enumerate(toks):
        om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
    ref = om.logits()
    got = st.logits()
    assert np.abs(got - ref).max() <= bar(ref), float(np.abs(got - ref).max())
    for layer in range(c.n_layers):
        for which in (0, 1):
            a = f16(gm.kv_read(layer, which, 0, len(toks)))
            b = f16(om.kv(layer, which)[:len(toks)])
            assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), (layer, which)


@pytest.mark.parametrize("heads,kv_heads", [(8, 2), (16, 2), (8, 8), (8, 4)])
def test_prompt_attention_shared_tiles_bit_identical(heads, kv_heads):
    """XH_OPT_PREFILL_ATTN 1 (K/V tiles DMA'd once per workgroup, ring in LDS, V read by
    transposed LDS reads) runs prefill_fa_kernel's per-wave arithmetic unchanged: logits and
    every K/V row of ragged prompts (a 333-token prompt, then 1000 tokens at pos 333, a pass
    boundary at 2048 crossed by 37 + 1400 more) are bit-identical to XH_OPT_PREFILL_ATTN 2."""
    c = make_cfg(256, 512, 2, heads, kv_heads, 128, 512, 4096)
    toks = [1] + [3 + (i * 53) % 500 for i in range(2769)]
    cuts = [0, 333, 1333, 2770]
    res = []
    for attn in (1, 2):
        gm, om = build_pair(c, L.F16)
        om.close()
        gm.set_option(L.OPT_PREFILL_ATTN, attn)
        gm.set_option(L.OPT_PREFILL_ATTN_SPLIT, 0)  # one walk of the history per workgroup, as mode 2
        st = InferenceState(c)
        for a, b in zip(cuts[:-1], cuts[1:]):
            gm.prefill(toks[a:b], a, st)
        kv = [gm.kv_read(layer, which, 0, len(toks)) for layer in range(c.n_layers) for which in (0, 1)]
        res.append((st.logits().copy(), kv))
        gm.close()
    assert np.array_equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("attn,split", [(1, 1), (1, 0), (2, 0), (0, 0)])
def test_prompt_over_long_history(attn, split):
    """A 200-token prompt pass at pos0 = 12000 over a synthetic 12000-slot KV history (8 KV heads x
    head_dim 128, 4 q per KV head): every token's attention walks ~375 K/V tiles through the
    shared-tile ring (1), the per-wave tiles (2) or the split-KV kernel (0).  Last logits and the
    pass's K/V rows against the oracle's token loop on the same weights and history."""
    c = make_cfg(256, 512, 2, 32, 8, 128, 512, 16384)
    gm, om = build_pair(c, L.F16)
    gm.set_option(L.OPT_PREFILL_ATTN, attn)
    gm.set_option(L.OPT_PREFILL_ATTN_SPLIT, split)  # 1: 56 workgroups -> 10 history splits each
    history, n = 12000, 200
    kv_dim = c.n_kv_heads * c.head_dim
    for layer in range(c.n_layers):
        for which in (0, 1):
            seed = 3100 + 2 * layer + which
            gm.kv_fill_synthetic(layer, which, 0, history, seed, 1.0)
            om.set_kv(layer, which, 0, O.synthetic(history, kv_dim, L.F16, seed, 0.0, 1.0))
    toks = [3 + (i * 29) % 500 for i in range(n)]
    st = InferenceState(c)
    gm.prefill(toks, history, st)
    for i, tok in enumerate(toks):
        om.forward(tok, history + i, L.OUTPUT_LOGITS if i == n - 1 else L.HYDRATE_KV_CACHE)
    ref = om.logits()
    assert np.abs(st.logits() - ref).max() <= bar(ref), float(np.abs(st.logits() - ref).max())
    for layer in range(c.n_layers):
        for which in (0, 1):
            a = f16(gm.kv_read(layer, which, history, n))
            b = f16(om.kv(layer, which)[history:history + n])
            assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), (layer, which)
    gm.close()
    om.close()


@pytest.mark.parametrize("n", [1, 2, 32, 256])
def test_short_prompt_over_32k_history(n):
    """Short prompt passes over a ~32.7k-slot history at configs[3]'s head shape (32 q heads, 8 KV
    heads, head_dim 128; src/main.cpp:94-100 resuming a long chat): a pass of n tokens has
    8 * ceil(n / 32) (KV head, query tile) workgroups, so XH_OPT_PREFILL_ATTN_SPLIT 1 walks the
    history in up to 64 splits merged in split order (n = 1 takes the decode step instead).  Both the split and the single-walk forms
    against the oracle's token loop (last logits, the pass's K/V rows), and the split form
    repeatable bit for bit (fixed merge order)."""
    c = make_cfg(256, 512, 2, 32, 8, 128, 512, 32768)
    gm, om = build_pair(c, L.F16)
    history = c.max_seq_len - 8 - n  # the pass ends inside the ring (no wrap: the batched path)
    kv_dim = c.n_kv_heads * c.head_dim
    for layer in range(c.n_layers):
        for which in (0, 1):
            seed = 3300 + 2 * layer + which
            gm.kv_fill_synthetic(layer, which, 0, history, seed, 1.0)
            om.set_kv(layer, which, 0, O.synthetic(history, kv_dim, L.F16, seed, 0.0, 1.0))
    toks = [3 + (i * 31) % 500 for i in range(n)]
    for i, tok in enumerate(toks):
        om.forward(tok, history + i, L.OUTPUT_LOGITS if i == n - 1 else L.HYDRATE_KV_CACHE)
    ref = om.logits()
    st = InferenceState(c)
    got = {}
    for split in (1, 0, 1):
        gm.set_option(L.OPT_PREFILL_ATTN_SPLIT, split)
        gm.prefill(toks, history, st)
        lg = st.logits().copy()
        assert np.abs(lg - ref).max() <= bar(ref), (split, float(np.abs(lg - ref).max()))
        for layer in range(c.n_layers):
            for which in (0, 1):
                a = f16(gm.kv_read(layer, which, history, n))
                b = f16(om.kv(layer, which)[history:history + n])
                assert np.abs(a - b).max() <= 2e-3 * max(1.0, np.abs(b).max()), (split, layer, which)
        if split in got:
            assert np.array_equal(lg.view(np.uint32), got[split].view(np.uint32))
        got[split] = lg
    gm.close()
    om.close()
