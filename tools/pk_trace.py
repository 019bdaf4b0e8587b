"""Persistent-engine timeline: per-phase durations and hand-off gaps for one decode token.

Runs the bench workload (synthetic weights) with tracing on and prints, per layer, the time
workgroup 0 spent in each phase (hand-off passed -> published) and waiting (published ->
next hand-off passed), averaged over layers, plus the token total.
"""
import argparse
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402

PH = ["qkv", "attn", "wo", "w13", "w2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="mistral-7b-f16")
    ap.add_argument("--tokens", type=int, default=16)
    args = ap.parse_args()
    w = bench.WORKLOADS[args.workload]
    c = bench.make_config(w)
    m = Model(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        m.upload_synthetic(kind, layer, dt, seed, mean, std)
    m.set_engine(1)
    st = InferenceState(c)
    prompt = bench.prompt_tokens(c.vocab_size)
    m.prefill(prompt, 0, st)
    m.decode_greedy(len(prompt), 4)
    m.debug_trace(1)
    m.decode_greedy(len(prompt) + 4, args.tokens)
    us = m.last_launch_us()
    tr = m.debug_trace(0).astype(np.int64)
    L = c.n_layers
    n = (L + 1) * 5 * 2 + 2
    print(f"launch {us:.1f} us for {args.tokens} tokens = {us / args.tokens:.1f} us/token")
    for wg, name in enumerate(["wg0", "wg_mid", "wg_last"]):
        t = tr[wg * n:(wg + 1) * n][: (L + 1) * 10].reshape(L + 1, 5, 2)
        t0 = t[L, 1, 1]
        if t0 == 0:
            print(name, "no trace")
            continue
        rel = lambda v: (v - t0) / 100.0  # noqa: E731  (100 MHz -> us)
        busy = {p: [] for p in PH}
        gaps = {p: [] for p in PH}
        for l in range(L):
            for p in range(5):
                a, b = t[l, p, 0], t[l, p, 1]
                if a and b:
                    busy[PH[p]].append((b - a) / 100.0)
            # waits: QKV published -> Wo passed (attention in between), Wo pub -> W13 passed, ...
            seq = [(l, 0, 1), (l, 2, 0), (l, 2, 1), (l, 3, 0), (l, 3, 1), (l, 4, 0)]
            for (la, pa, ka), (lb, pb, kb) in zip(seq[0::2], seq[1::2]):
                if t[la, pa, ka] and t[lb, pb, kb]:
                    gaps[PH[pb]].append((t[lb, pb, kb] - t[la, pa, ka]) / 100.0)
            if l + 1 < L and t[l, 4, 1] and t[l + 1, 0, 0]:
                gaps["qkv"].append((t[l + 1, 0, 0] - t[l, 4, 1]) / 100.0)
        end = t[L, 1, 0] or t[L, 0, 1]
        print(f"{name}: token {rel(end):.1f} us; cls passed {rel(t[L, 0, 0]):.1f} published {rel(t[L, 0, 1]):.1f}")
        for p in PH:
            bb, gg = busy[p], gaps[p]
            print(f"  {p:5s} busy {np.mean(bb) if bb else float('nan'):7.2f} us (n={len(bb)})"
                  f"  wait-before {np.mean(gg) if gg else float('nan'):7.2f} us")
    m.close()


if __name__ == "__main__":
    main()
