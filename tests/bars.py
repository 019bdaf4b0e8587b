"""Logits bars of the GPU-vs-oracle parity tests.

The north-star bar is 1e-3 max-abs (BASELINE.json), stated relative to the logit scale above 1
(small_llama's logits reach |93|).  On the converter fixtures the bar is tighter: MARGIN x the
measured envelope of that fixture and path (tests/golden/error_envelope.json: the largest error
any GPU test saw, written by tools/error_envelope.py from a run with XALM_ERR_LOG set), capped
by the north-star bar — so a systematic error of a few ulps of the logit scale fails instead of
hiding under 1e-3 x 93.  Paths: "loop" (token-by-token forward / device greedy loop), "prefill"
(the batched MFMA prompt passes), "ppl" (log-probabilities of xh_perplexity).
"""
import json
import os

import numpy as np

MARGIN = 8.0
_ENV_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "error_envelope.json")
ENVELOPE = json.load(open(_ENV_PATH)) if os.path.exists(_ENV_PATH) else {}
_LOG = []  # (test id, fixture, path, err, scale) when XALM_ERR_LOG is set (conftest writes it)


def north(ref):
    return 1e-3 * max(1.0, float(np.abs(ref).max()))


def bar(ref, fixture=None, path="loop"):
    b = north(ref)
    env = ENVELOPE.get(fixture or "", {}).get(path)
    return min(b, MARGIN * env) if env else b


def record(fixture, path, err, scale):
    if os.environ.get("XALM_ERR_LOG"):
        _LOG.append((os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], fixture, path, err, scale))


def check(got, ref, fixture=None, path="loop", what=""):
    """assert max|got - ref| <= bar; the error is logged for the envelope."""
    err = float(np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64)).max())
    record(fixture, path, err, float(np.abs(ref).max()))
    b = bar(ref, fixture, path)
    assert err <= b, (fixture, path, what, err, b)
    return err


def check_logp(err, logits, fixture=None, what=""):
    """|log p - log p_ref| of one scored token (xh_perplexity): at most 2x the logits bar of that
    position (+1e-5), or MARGIN x the fixture's measured "ppl" envelope."""
    record(fixture, "ppl", err, 1.0)
    b = 2 * north(logits) + 1e-5
    env = ENVELOPE.get(fixture or "", {}).get("ppl")
    if env:
        b = min(b, MARGIN * env)
    assert err <= b, (fixture, what, err, b)
