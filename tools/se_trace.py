#!/usr/bin/env python
"""Stream-engine timeline (xh_debug_trace bit 8) on the Mistral-7B bench shapes.

Runs one decode_greedy launch of N tokens with tracing on and prints, for the last token of
CUs {0, n/2, n-1}, per phase: wait for the phase input (hand-off), matrix time, and when the
loader issued the phase's first slot; plus chip-wide stall sums per CU (median / max).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="mistral-7b-f16")
ap.add_argument("--tokens", type=int, default=8)
ap.add_argument("--layers", type=int, default=0, help="override layer count (0 = workload's)")
ap.add_argument("--ncu", type=int, default=256, help="CUs of the device (MI355X: 256)")
args = ap.parse_args()
w = dict(bench.WORKLOADS[args.workload])
if args.layers:
    w["layers"] = args.layers
c = bench.make_config(w)
m = Model(c)
for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
    m.upload_synthetic(kind, layer, dt, seed, mean, std)
m.set_engine(2)
st = InferenceState(c)
prompt = bench.prompt_tokens(c.vocab_size)
m.prefill(prompt, 0, st)
m.decode_greedy(len(prompt), 4)
n = m.debug_trace(8)
m.decode_greedy(len(prompt) + 4, args.tokens)
us = m.last_launch_us()
tr = m.debug_trace(0)
L_ = c.n_layers
nph = 4 * L_ + 1  # 4 phases per layer + the lm_head (every decode token has logits)
print(f"launch {us:.0f} us for {args.tokens} tokens = {us / args.tokens:.1f} us/token")
ncu = args.ncu
raw = np.array(tr[:8 * ncu], dtype=np.float64).reshape(ncu, 8)
sums = raw / 100.0  # us
names = ["loader ring-full", "wave0 ring-empty", "wave0 hand-off", "wave0 attention"]
for k in range(4):
    print(f"  {names[k]:18s}: median {np.median(sums[:, k]) / args.tokens:8.1f} us/token  max {sums[:, k].max() / args.tokens:8.1f}")
lat = sums[:, 4] / np.maximum(raw[:, 5], 1)
print(f"  loader issue->landed per slot: median {np.median(lat):6.2f} us  max {lat.max():6.2f} us; "
      f"vmcnt-blocked median {np.median(sums[:, 6]) / args.tokens:8.1f} us/token")
base = 8 * ncu
ph_names = ["qkv", "wo", "w13", "w2"]
for k, cu in enumerate(("cu0", "cu_mid", "cu_last")):
    s = np.array(tr[base + k * nph * 8: base + (k + 1) * nph * 8], dtype=np.int64).reshape(nph, 8)
    if not s[0, 0]:
        continue
    t0 = s[0, 0]
    print(f"{cu}: per phase (us from token start): [input wait start, ready, matrix done, loader first issue,"
          " attention: qkv counted, K/V loaded, published]")
    for q in range(nph):
        name = "cls" if q == 4 * L_ else f"l{q // 4}.{ph_names[q % 4]}"
        if q < 8 or q >= nph - 5:
            print(f"  {name:8s} " + " ".join(f"{(v - t0) / 100.0:9.1f}" if v else "        -" for v in s[q][:7]))
    ready = (s[:, 1] - s[:, 0]) / 100.0
    mat = (s[:, 2] - s[:, 1]) / 100.0
    for p in range(4):
        print(f"  {ph_names[p]}: input wait avg {ready[p:4 * L_:4].mean():6.2f} us, matrix avg {mat[p:4 * L_:4].mean():6.2f} us")
m.close()
