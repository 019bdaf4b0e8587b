"""Generate the gguf-block fixtures (Q8_0 / Q4_0) under tests/golden/.

* ``tiny_mistral_q8_0.xalm``, ``tiny_mistral_q4_0.xalm``, ``small_llama_q8_0.xalm``: the
  same synthetic checkpoints as make_fixtures.py, written by the REFERENCE converter
  (convert.py ``--type q8_0 / q4_0``: XType.convert_to :176-187 -> quants.py ``quantize``),
  executed from /root/reference in memory exactly as make_fixtures.py does.
* ``gq_golden.npz``: inputs (seeded float32 rows plus edge rows: zeros, ties of the largest
  magnitude, a negative maximum, values near the rounding boundaries) with the bytes of
  quants.py ``quantize`` and the floats of quants.py ``dequantize`` for Q8_0 and Q4_0.  They
  pin the oracle's block decode and the shared quantizer (include/xalm_synth.h) bit for bit.

Run:  python tests/golden/make_gq_fixtures.py      (needs /root/reference, torch)
"""
from __future__ import annotations

import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_fixtures as mf  # noqa: E402


def gq_inputs():
    rng = np.random.default_rng(2024)
    rows = [rng.normal(0.0, 0.02, 256).astype(np.float32) for _ in range(6)]
    rows.append(np.zeros(256, np.float32))
    tie = rng.normal(0.0, 0.02, 256).astype(np.float32)
    tie[3], tie[17] = 0.05, -0.05          # equal magnitudes: argmax takes the first
    tie[40], tie[50] = -0.07, 0.07
    rows.append(tie)
    neg = rng.normal(0.0, 1.0, 256).astype(np.float32)
    neg[5] = -9.0                          # a negative maximum magnitude (Q4_0 d > 0)
    rows.append(neg)
    half = (np.arange(256, dtype=np.float32) % 32 - 15.5) * np.float32(1.0 / 127.0)
    rows.append(half)                      # products near .5 after scaling
    big = rng.normal(0.0, 300.0, 256).astype(np.float32)
    rows.append(big)
    tiny = rng.normal(0.0, 1e-6, 256).astype(np.float32)
    rows.append(tiny)                      # f16 subnormal scales
    return np.stack(rows)


def main():
    sys.path.insert(0, mf.REF)
    import quants  # the reference's quantizer (imported from /root/reference, not copied)

    x = gq_inputs()
    out = {"inputs": x}
    for name, qt in (("q8_0", quants.GGMLQuantizationType.Q8_0), ("q4_0", quants.GGMLQuantizationType.Q4_0)):
        q = quants.quantize(x, qt)
        out[name] = np.ascontiguousarray(q, dtype=np.uint8)
        out[name + "_deq"] = np.ascontiguousarray(quants.dequantize(q, qt), dtype=np.float32)
    np.savez_compressed(os.path.join(HERE, "gq_golden.npz"), **out)
    print("wrote gq_golden.npz", {k: v.shape for k, v in out.items()})

    import torch  # noqa: F401
    conv = mf.load_reference_converter()
    for name, types in (("tiny_mistral", ["q8_0", "q4_0"]), ("small_llama", ["q8_0"])):
        spec = mf.MODELS[name]
        tmp = tempfile.mkdtemp(prefix=f"xalm_gq_{name}_")
        try:
            mf.write_checkpoint(tmp, spec)
            for t in types:
                path = os.path.join(HERE, f"{name}_{t}.xalm")
                mf.convert(conv, tmp, path, t)
                print("wrote", path, os.path.getsize(path))
        finally:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
