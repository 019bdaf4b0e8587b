"""Diagnostic (not collected by pytest): prefill logits across XH_OPT_PREFILL modes and the GLU-split knob, repeated, vs the oracle."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.dirname(__file__))
import numpy as np
from xalm_amd import _lib as L
from xalm_amd.model import InferenceState
from test_forward_gpu import synthetic_pair

toks = [1] + [3 + (i * 37) % 500 for i in range(99)]
for wdt in (L.F8_E4M3, L.F16):
    ref = None
    for mode in (1, 2):
        for glu in (1, 0, 1, 0):
            gm, om = synthetic_pair(wdt)
            if ref is None:
                for pos, tok in enumerate(toks):
                    om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
                ref = om.logits().copy()
            gm.set_option(L.OPT_PREFILL, mode)
            gm.set_option(L.OPT_PREFILL_GLU_SPLIT, glu)
            st = InferenceState(gm.config)
            gm.prefill(toks, 0, st)
            lg = st.logits()
            print(f"wdt {wdt} mode {mode} glu {glu}: max|d| vs oracle {np.abs(lg - ref).max():.3e} sum {lg.sum():.6f}", flush=True)
            gm.close()
