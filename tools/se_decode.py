#!/usr/bin/env python
"""A short Mistral-7B-shaped decode on one engine (for rocprofv3 counter passes)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--engine", type=int, default=2)
ap.add_argument("--tokens", type=int, default=8)
ap.add_argument("--workload", default="mistral-7b-f16")
args = ap.parse_args()
w = bench.WORKLOADS[args.workload]
c = bench.make_config(w)
m = Model(c)
for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
    m.upload_synthetic(kind, layer, dt, seed, mean, std)
m.set_engine(args.engine)
st = InferenceState(c)
prompt = bench.prompt_tokens(c.vocab_size)
m.prefill(prompt, 0, st)
toks = m.decode_greedy(len(prompt), args.tokens)
print("engine", m.engine, "tokens", toks[:8])
m.close()
