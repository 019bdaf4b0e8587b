"""Full-size parity of every BASELINE GPU config against the reference algorithm's exact value.

The north-star bar is "logits within 1e-3 max-abs of the CPU reference" (src/infer.cpp:604-638).
At full size (32 layers of random weights) the reference's OWN f32 result is not that close to the
algorithm's exact value: a 32-layer network amplifies f32 rounding (and the fp16 K/V roundings it
flips), so two valid f32 evaluations — the 8-wide FMA lanes and the sequential reading of the
reference's `omp simd` row loop (src/infer.cpp:104-135) — differ from each other by ~3e-3.  The
precision-independent check: evaluate the same algorithm in double (oracle
xo_set_precision(m, 1): every product, sum, norm, softmax, activation and residual in f64; the fp16
K/V cache and the float rope angles kept as the reference defines them) and require the GPU to be
at least as close to that value as the reference's own f32 loop is:

    max|GPU - oracle64| <= max over both f32 orders of max|oracle32 - oracle64|

for the batched prompt path, the token-by-token path and the device greedy loop, plus argmax
agreement with oracle64 wherever its top-2 margin exceeds twice that spread.  Workloads are
bench.py's (BASELINE configs[1..4]: Mistral-7B f16 4k (two weight seeds), fp8 e4m3 with bf16
embed / lm_head, -T 32768 with a full ring and the StreamingLLM sinks, Llama-3-8B V = 128256; and
the SURVEY 8f-4 gguf Q8_0 / Q4_0 block workloads, quants.py:281-465), synthetic weights generated
bit-identically on the device and the host (include/xalm_synth.h).  The 32k ring is also checked
through a batched prompt pass over a 32700-slot history (test_long_history_prompt_pass).
"""
import json
import os
import time

import numpy as np
import pytest

import bench
from oracle import oracle as O
from xalm_amd import _lib as L
from xalm_amd.model import InferenceState, Model

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

DECODE = 16  # device greedy steps after the prompt (32k: after the one-token hydrate)


def maxabs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def gpu_side(w, c, shift=0):
    """GPU logits: batched prompt, token loop, and DECODE device greedy steps after the loop."""
    gm = Model(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w, shift):
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
    prompt = bench.prompt_tokens(c.vocab_size)
    st = InferenceState(c)
    out = {}
    if w["kv_prefill"]:
        hist = w["kv_prefill"]

        def fill():
            for layer in range(c.n_layers):
                gm.kv_fill_synthetic(layer, 0, 0, hist, 5000 + 2 * layer, 1.0)
                gm.kv_fill_synthetic(layer, 1, 0, hist, 5001 + 2 * layer, 1.0)
        fill()
        gm.forward(st, prompt[0], hist, L.OUTPUT_LOGITS)
        out["loop"] = st.logits().copy()
        toks = gm.decode_greedy(hist + 1, DECODE)
        gm.get_logits(st)
        out["decode"] = st.logits().copy()
        out["tokens"] = list(toks)
        out["hydrate"] = prompt[:1]
        out["pos0"] = hist
    else:
        gm.prefill(prompt, 0, st)
        out["prefill"] = st.logits().copy()
        gm.reset()
        for pos, tok in enumerate(prompt):
            gm.forward(st, tok, pos, L.OUTPUT_LOGITS if pos == len(prompt) - 1 else L.HYDRATE_KV_CACHE)
        out["loop"] = st.logits().copy()
        toks = gm.decode_greedy(len(prompt), DECODE)
        gm.get_logits(st)
        out["decode"] = st.logits().copy()
        out["tokens"] = list(toks)
        out["hydrate"] = prompt
        out["pos0"] = 0
    gm.close()
    return out


def oracle_side(w, c, g, weights, kv):
    """(logits after the hydrate, logits after the GPU's DECODE tokens) for oracle64 and the two
    f32 orders; teacher-forced on the GPU's tokens so every variant sees the same inputs."""
    res = {}
    for name, prec, order in (("o64", 1, 0), ("lanes", 0, 0), ("seq", 0, 1)):
        if name == "seq" and w["wdt"] not in (L.F16, L.F8_E4M3, L.F8_E5M2, L.Q8_0, L.Q4_0):
            continue  # bf16 matmuls have one (sequential) order only: lanes == seq
        O.set_matmul_order(order)
        om = O.OracleModel(c)
        try:
            for kind, layer, dt, arr in weights:
                om.set_tensor(kind, layer, dt, arr)
            for layer, which, arr in kv:
                om.set_kv(layer, which, 0, arr)
            om.set_precision(prec)
            t0 = time.time()
            hyd, pos0 = g["hydrate"], g["pos0"]
            for i, tok in enumerate(hyd):
                om.forward(tok, pos0 + i, L.OUTPUT_LOGITS if i == len(hyd) - 1 else L.HYDRATE_KV_CACHE)
            first = om.logits()
            pos = pos0 + len(hyd)
            for i, tok in enumerate(g["tokens"]):
                om.forward(tok, pos + i, L.OUTPUT_LOGITS)
            res[name] = (first, om.logits(), time.time() - t0)
        finally:
            om.close()
            O.set_matmul_order(0)
    return res


def check_report(rep, g, o, checks):
    """GPU within the reference f32 evaluation's distance from oracle64 on every path, argmax
    agreement outside near-ties; the report goes to stdout and XALM_PARITY_OUT (jsonl)."""
    exact0, exactN = o["o64"][0], o["o64"][1]
    f32 = [k for k in ("lanes", "seq") if k in o]
    spread0 = max(maxabs(o[k][0], exact0) for k in f32)
    spreadN = max(maxabs(o[k][1], exactN) for k in f32)
    rep.update({"logit_scale": float(np.abs(exact0).max()),
                "oracle32_vs_oracle64": {k: [maxabs(o[k][0], exact0), maxabs(o[k][1], exactN)] for k in f32},
                "gpu_vs_oracle64": {}, "gpu_vs_oracle32_lanes": {},
                "oracle_seconds": {k: round(v[2], 1) for k, v in o.items()}, "gpu_tokens": g.get("tokens", [])})
    for path, idx in checks:
        if path not in g:
            continue
        rep["gpu_vs_oracle64"][path] = maxabs(g[path], o["o64"][idx])
        rep["gpu_vs_oracle32_lanes"][path] = maxabs(g[path], o["lanes"][idx])
    print(json.dumps(rep))
    out = os.environ.get("XALM_PARITY_OUT")
    if out:
        with open(out, "a") as f:
            f.write(json.dumps(rep) + "\n")
    for path, idx in checks:
        if path not in g:
            continue
        bound = spread0 if idx == 0 else spreadN
        assert rep["gpu_vs_oracle64"][path] <= bound, (path, rep["gpu_vs_oracle64"][path], bound)
        exact = o["o64"][idx]
        top2 = np.sort(exact)[-2:]
        if top2[1] - top2[0] > 2 * bound:
            assert int(np.argmax(g[path])) == int(np.argmax(exact)), path


# (workload, weight seed shift): the BASELINE GPU configs, a second draw of configs[1], and the
# gguf block workloads (their oracle decodes every block element as quants.py dequantizes it)
CASES = [("mistral-7b-f16", 0), ("mistral-7b-f16", 7919), ("mistral-7b-f8", 0), ("llama3-8b-f16", 0),
         ("mistral-7b-f16-32k", 0), ("mistral-7b-q8_0", 0), ("mistral-7b-q4_0", 0)]


@pytest.mark.parametrize("workload,shift", CASES, ids=[f"{w}-seed{s}" for w, s in CASES])
def test_full_size_within_reference_f32_error_of_exact(workload, shift):
    w = bench.WORKLOADS[workload]
    c = bench.make_config(w)
    g = gpu_side(w, c, shift)
    weights = [(kind, layer, dt, O.synthetic(*bench.tensor_shape(c, kind), dt, seed, mean, std))
               for kind, layer, dt, seed, mean, std in bench.tensor_specs(w, shift)]
    kv = []
    if w["kv_prefill"]:
        kv_dim = c.n_kv_heads * c.head_dim
        kv = [(layer, which, O.synthetic(w["kv_prefill"], kv_dim, L.F16, 5000 + 2 * layer + which, 0.0, 1.0))
              for layer in range(c.n_layers) for which in (0, 1)]
    o = oracle_side(w, c, g, weights, kv)
    del weights, kv
    check_report({"workload": workload, "seed_shift": shift, "decode_steps": DECODE}, g, o,
                 [("prefill", 0), ("loop", 0), ("decode", 1)])
    # the device greedy tokens: each is oracle64's argmax at its step unless that step is a near-tie
    # (checked through the final logits above; the teacher-forced tokens are the GPU's own)


@pytest.mark.parametrize("workload", ["mistral-7b-f16", "mistral-7b-f8"])
def test_full_size_2048_token_pass_glu_epilogues_agree(workload):
    """A 2048-token prompt pass at Mistral-7B shapes (the W1/W3 GEMM on the 4-wave launch):
    act(g) * u (src/infer.cpp:468-488) fused with the W2 input split (prefill_glu_split_kernel)
    gives the same logits, bit for bit, as the GLU epilogue kernel + separate split
    (XH_OPT_PREFILL_GLU_SPLIT 0)."""
    w = bench.WORKLOADS[workload]
    c = bench.make_config(w)
    gm = Model(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
    prompt = bench.prompt_tokens(c.vocab_size, n=2048, seed=11)
    st = InferenceState(c)
    got = {}
    for glu in (1, 0):
        gm.reset()
        gm.set_option(L.OPT_PREFILL_GLU_SPLIT, glu)
        gm.prefill(prompt, 0, st)
        got[glu] = st.logits().copy()
    assert np.isfinite(got[1]).all()
    assert np.array_equal(got[1].view(np.uint32), got[0].view(np.uint32))


# configs[3]'s ring through the batched prompt path, in three tests (each well under the runner's
# silence limit; pytest -x runs them in order and they share _P32): a 32700-slot synthetic history,
# one 32-token prompt pass at pos0 = 32700 (no wrap: prefill.h's MFMA prompt attention over the
# whole history; the reference hydrates token by token, src/infer.cpp:604-638 / src/main.cpp:94-100),
# logits of its last token, then DECODE_32K device greedy steps (the split-KV decode attention at
# 32.7k slots).  Oracle: the fp64 evaluation and both f32 orders.
_P32 = {}
DECODE_32K = 6


def _p32_setup():
    if "w" not in _P32:
        w = bench.WORKLOADS["mistral-7b-f16-32k"]
        c = bench.make_config(w)
        hist, n = 32700, 32
        _P32.update(w=w, c=c, hist=hist, prompt=bench.prompt_tokens(c.vocab_size, n=n, seed=13))
    return _P32


def test_long_history_prompt_pass_gpu():
    p = _p32_setup()
    w, c, hist, prompt = p["w"], p["c"], p["hist"], p["prompt"]
    gm = Model(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        gm.upload_synthetic(kind, layer, dt, seed, mean, std)
    for layer in range(c.n_layers):
        gm.kv_fill_synthetic(layer, 0, 0, hist, 5000 + 2 * layer, 1.0)
        gm.kv_fill_synthetic(layer, 1, 0, hist, 5001 + 2 * layer, 1.0)
    st = InferenceState(c)
    gm.prefill(prompt, hist, st)
    g = {"prefill": st.logits().copy(), "hydrate": prompt, "pos0": hist}
    g["tokens"] = list(gm.decode_greedy(hist + len(prompt), DECODE_32K))
    gm.get_logits(st)
    g["decode"] = st.logits().copy()
    gm.close()
    p["g"] = g


def _p32_oracle(name, prec, part, order=0):
    """one evaluation in two parts (each test stays short): part 0 builds the oracle and hydrates
    the first half of the prompt; part 1 the rest of the prompt and the GPU's greedy tokens"""
    p = _p32_setup()
    assert "g" in p, "runs after test_long_history_prompt_pass_gpu"
    w, c, hist, g = p["w"], p["c"], p["hist"], p["g"]
    hyd = g["hydrate"]
    half = len(hyd) // 2
    O.set_matmul_order(order)
    if part == 0:
        kv_dim = c.n_kv_heads * c.head_dim
        om = O.OracleModel(c)
        for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
            om.set_tensor(kind, layer, dt, O.synthetic(*bench.tensor_shape(c, kind), dt, seed, mean, std))
        for layer in range(c.n_layers):
            for which in (0, 1):
                om.set_kv(layer, which, 0, O.synthetic(hist, kv_dim, L.F16, 5000 + 2 * layer + which, 0.0, 1.0))
        om.set_precision(prec)
        p["om"], p["t"] = om, 0.0
        t0 = time.time()
        for i in range(half):
            om.forward(hyd[i], hist + i, L.HYDRATE_KV_CACHE)
        p["t"] += time.time() - t0
        O.set_matmul_order(0)
        return
    om = p.pop("om")
    try:
        t0 = time.time()
        for i in range(half, len(hyd)):
            om.forward(hyd[i], hist + i, L.OUTPUT_LOGITS if i == len(hyd) - 1 else L.HYDRATE_KV_CACHE)
        first = om.logits()
        pos = hist + len(hyd)
        for i, tok in enumerate(g["tokens"]):
            om.forward(tok, pos + i, L.OUTPUT_LOGITS)
        p[name] = (first, om.logits(), p["t"] + time.time() - t0)
    finally:
        om.close()
        O.set_matmul_order(0)


def test_long_history_prompt_pass_oracle64_a():
    _p32_oracle("o64", 1, 0)


def test_long_history_prompt_pass_oracle64_b():
    _p32_oracle("o64", 1, 1)


def test_long_history_prompt_pass_oracle32_lanes_a():
    _p32_oracle("lanes", 0, 0)


def test_long_history_prompt_pass_oracle32_lanes_b():
    _p32_oracle("lanes", 0, 1)


def test_long_history_prompt_pass_oracle32_seq_a():
    _p32_oracle("seq", 0, 0, order=1)


def test_long_history_prompt_pass_vs_oracle():
    _p32_oracle("seq", 0, 1, order=1)
    p = _P32
    o = {"o64": p["o64"], "lanes": p["lanes"], "seq": p["seq"]}
    check_report({"workload": "mistral-7b-f16-32k prompt pass", "pos0": p["hist"], "prompt_tokens": len(p["prompt"]),
                  "decode_steps": DECODE_32K}, p["g"], o, [("prefill", 0), ("decode", 1)])
