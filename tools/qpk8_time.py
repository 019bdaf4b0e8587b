#!/usr/bin/env python
"""Decode step time of a GQA-8 model (32 q heads x 128 over 4 KV heads, Mistral-7B's other
shapes, 8 layers) with attention + Wo fused in one launch (XH_OPT_FUSE_ATTN_WO 1) or as two
launches (0): the fused kernel's QPK = 8 instantiation is register-bound."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402

w = dict(bench.WORKLOADS["mistral-7b-f16"], layers=8, kv_heads=4)
c = bench.make_config(w)
m = Model(c)
for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
    m.upload_synthetic(kind, layer, dt, seed, mean, std)
st = InferenceState(c)
prompt = bench.prompt_tokens(c.vocab_size)
for fuse in (1, 0, 1, 0):
    m.set_option(L.OPT_FUSE_ATTN_WO, fuse)
    m.reset()
    m.prefill(prompt, 0, st)
    m.decode_greedy(len(prompt), 8)
    t = time.perf_counter()
    m.decode_greedy(len(prompt) + 8, 128)
    dt = (time.perf_counter() - t) / 128
    print(f"fuse {fuse}: {dt * 1e3:.4f} ms per token (8 layers, QPK 8), attention {m.time_kernel(5, 50):.2f} us", flush=True)
m.close()
