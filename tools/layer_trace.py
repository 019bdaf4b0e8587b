"""Timeline of the last layer's launches + lm_head inside the decode graph (device clock, 100 MHz):
per launch the first / last workgroup start, median x staged, first / median / last end, and the
boundary from one launch's last workgroup end to the next launch's first workgroup start."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402

# (name, first word, words, words per workgroup): xalm_hip.hip LT_* regions
REGIONS = [("qkv", 0, 8192, 4), ("attn+wo", 8192, 8192, 8), ("w1/w3", 16384, 4096, 4), ("w2", 20480, 4096, 4),
           ("lm_head", 24576, 4096, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="mistral-7b-f16")
    ap.add_argument("--opt", action="append", default=[], help="NAME=VALUE of an XH_OPT_* (e.g. FUSE_ATTN_WO=0)")
    args = ap.parse_args()
    w = bench.WORKLOADS[args.workload]
    c = bench.make_config(w)
    m = Model(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        m.upload_synthetic(kind, layer, dt, seed, mean, std)
    for o in args.opt:
        k, v = o.split("=")
        m.set_option(getattr(L, "OPT_" + k), int(v))
    st = InferenceState(c)
    prompt = bench.prompt_tokens(c.vocab_size)
    if w["kv_prefill"]:
        # configs[3]: a filled 32k ring, decode right after it (kv_len = max_seq_len)
        for layer in range(c.n_layers):
            m.kv_fill_synthetic(layer, 0, 0, w["kv_prefill"], 5000 + 2 * layer, 1.0)
            m.kv_fill_synthetic(layer, 1, 0, w["kv_prefill"], 5001 + 2 * layer, 1.0)
        pos = w["kv_prefill"]
        m.prefill(prompt[:1], pos, st)
        pos += 1
    else:
        m.prefill(prompt, 0, st)
        pos = len(prompt)
    m.decode_greedy(pos, 20)
    m.debug_trace(16)
    m.decode_greedy(pos + 20, 3)
    tr = m.debug_trace(0).astype(np.int64)
    spans = []
    t0 = None
    for name, off, words, stride in REGIONS:
        t = tr[off: off + words]
        t = t[: t.size // stride * stride].reshape(-1, stride)
        used = t[:, 0] != 0
        t = t[used]
        if not t.size:
            continue
        if t0 is None:
            t0 = t[:, 0].min()
        us = lambda v: (v - t0) / 100.0  # noqa: E731
        s0, s1 = us(t[:, 0].min()), us(t[:, 0].max())
        end = t[:, 2][t[:, 2] != 0]
        stg = t[:, 1][t[:, 1] != 0]
        e = us(end) if end.size else np.array([np.nan])
        if os.environ.get("XLANDED") and stride == 4:
            xl = t[:, 3][(t[:, 3] != 0) & (t[:, 3] > t[:, 0].min())]
            if xl.size:
                q = np.percentile(us(xl), [10, 50, 90])
                print(f"{name:8s} x landed p10 {q[0]:7.2f} med {q[1]:7.2f} p90 {q[2]:7.2f}")
        print(f"{name:8s} wgs {t.shape[0]:4d}  start {s0:7.2f}..{s1:7.2f}  staged med {np.median(us(stg)) if stg.size else float('nan'):7.2f}"
              f"  end min {np.min(e):7.2f} med {np.median(e):7.2f} max {np.max(e):7.2f}  span {np.max(e) - s0:6.2f} us")
        spans.append((name, s0, np.max(e)))
    for (a, _, ea), (b, sb, _) in zip(spans, spans[1:]):
        print(f"  boundary {a} -> {b}: {sb - ea:5.2f} us")
    m.close()


if __name__ == "__main__":
    main()
