#!/usr/bin/env python
"""Short prompt passes over a full -T 32768 ring (configs[3] shapes, synthetic weights and K/V
history): xh_prefill of N tokens at pos0 = 32768 - N, REPEAT times, with the prompt attention's
history splits on or off.  For rocprofv3 kernel stats of the prompt attention in this regime:
    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/short_pass.py 1 --split 1
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="+")
ap.add_argument("--split", type=int, default=1)
ap.add_argument("--repeat", type=int, default=3)
args = ap.parse_args()
w = bench.WORKLOADS["mistral-7b-f16-32k"]
c = bench.make_config(w)
m = Model(c)
for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
    m.upload_synthetic(kind, layer, dt, seed, mean, std)
for layer in range(c.n_layers):
    m.kv_fill_synthetic(layer, 0, 0, c.max_seq_len, 5000 + 2 * layer, 1.0)
    m.kv_fill_synthetic(layer, 1, 0, c.max_seq_len, 5001 + 2 * layer, 1.0)
m.set_option(L.OPT_PREFILL_ATTN_SPLIT, args.split)
st = InferenceState(c)
for n in args.n:
    toks = bench.prompt_tokens(c.vocab_size, n=n, seed=17)
    ts = []
    for _ in range(args.repeat):
        t0 = time.perf_counter()
        m.prefill(toks, c.max_seq_len - n, st)
        ts.append(1e3 * (time.perf_counter() - t0))
    print(f"n {n} split {args.split}: ms per pass {' '.join(f'{t:.3f}' for t in ts)}", flush=True)
m.close()
