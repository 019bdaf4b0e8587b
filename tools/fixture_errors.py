"""Measured GPU-vs-oracle logit errors on the converter fixtures, per scenario (the envelope the
fixture tests' bars are set from; tests/test_forward_gpu.py ERR_BAR)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import fixture_path  # noqa: E402
from oracle import oracle as O  # noqa: E402
from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402
from xalm_amd.xalm_file import XalmFile  # noqa: E402

FIXTURES = ["tiny_mistral_f16", "tiny_mistral_bf16", "tiny_mistral_f32", "tiny_mistral_f8_e4m3",
            "tiny_mistral_f8_e5m2", "small_llama_f16", "tiny_mistral_q8_0", "tiny_mistral_q4_0", "small_llama_q8_0"]


def main():
    for name in FIXTURES:
        xf = XalmFile(fixture_path(name + ".xalm"))
        res = {}
        # token loop, both launch structures, 24 positions
        for fuse in (1, 0):
            gm, om = Model.from_xalm(xf), O.OracleModel.from_xalm(xf)
            gm.set_option(L.OPT_FUSE_ATTN_WO, fuse)
            st = InferenceState(gm.config)
            worst, scale = 0.0, 0.0
            for pos in range(24):
                tok = 1 if pos == 0 else 3 + (pos * 37) % (gm.config.vocab_size - 3)
                gm.forward(st, tok, pos)
                om.forward(tok, pos)
                worst = max(worst, float(np.abs(st.logits() - om.logits()).max()))
                scale = max(scale, float(np.abs(om.logits()).max()))
            res[f"loop fuse{fuse}"] = worst
            gm.close()
            om.close()
        # ring wrap at -T 16
        gm, om = Model.from_xalm(xf, context=16), O.OracleModel.from_xalm(xf, context=16)
        st = InferenceState(gm.config)
        w = 0.0
        for pos in range(40):
            tok = 1 if pos == 0 else 3 + (pos * 37) % (gm.config.vocab_size - 3)
            gm.forward(st, tok, pos)
            om.forward(tok, pos)
            w = max(w, float(np.abs(st.logits() - om.logits()).max()))
        res["ring -T16"] = w
        # batched prefill, every GEMM mode (block formats take the token loop)
        for mode in (1, 2, 3):
            gm, om = Model.from_xalm(xf, context=256), O.OracleModel.from_xalm(xf, context=256)
            gm.set_option(L.OPT_PREFILL, mode)
            toks = [1] + [3 + (i * 37) % 280 for i in range(99)]
            st = InferenceState(gm.config)
            gm.prefill(toks, 0, st)
            for pos, tok in enumerate(toks):
                om.forward(tok, pos, L.OUTPUT_LOGITS if pos == len(toks) - 1 else L.HYDRATE_KV_CACHE)
            res[f"prefill {mode}"] = float(np.abs(st.logits() - om.logits()).max())
            gm.close()
            om.close()
        print(f"{name:22s} logit scale {scale:7.3f}  " + "  ".join(f"{k} {v:.2e}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
