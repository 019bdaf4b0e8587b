"""Timeline of one fused qkv + attention + Wo launch (qaw.h): the last layer of the last
decoded token, per workgroup role, in microseconds from the launch's first stamp."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="mistral-7b-f16")
    ap.add_argument("--decode", type=int, default=200)
    args = ap.parse_args()
    w = bench.WORKLOADS[args.workload]
    c = bench.make_config(w)
    m = Model(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        m.upload_synthetic(kind, layer, dt, seed, mean, std)
    st = InferenceState(c)
    prompt = bench.prompt_tokens(c.vocab_size)
    m.prefill(prompt, 0, st)
    m.decode_greedy(len(prompt), args.decode)
    print("fuse level in effect:", m.get_option(L.OPT_FUSE_ATTN_WO))
    m.debug_trace(4)
    m.decode_greedy(len(prompt) + args.decode, 2)
    tr = m.debug_trace(0).astype(np.int64)
    n = tr.size // 8
    t = tr[: n * 8].reshape(n, 8)
    used = np.nonzero(t[:, 0])[0]
    if used.size == 0:
        print("no stamps")
        return
    t0 = t[used, 0].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731
    nsplit = min(16, max(1, min(512 // c.n_kv_heads, 128, (c.max_seq_len + 255) // 256)))
    natt = c.n_kv_heads * nsplit
    att = [i for i in used if i < natt]
    rows = [i for i in used if i >= natt]
    print(f"workgroups traced: {len(used)} (attention {len(att)}, rows {len(rows)})")

    def show(name, ids, k):
        v = np.array([us(t[i, k]) for i in ids if t[i, k]])
        if v.size:
            print(f"  {name:22s} n {v.size:4d} min {v.min():7.2f} med {np.median(v):7.2f} max {v.max():7.2f} us")

    print("attention workgroups")
    show("start", att, 0)
    show("qkv hand-off passed", att, 1)
    for k, name in ((2, "split known"), (3, "scores done"), (6, "softmax done"), (7, "p.V summed"), (4, "p.V reduced"),
                    (5, "partial drained")):
        show(name, [i for i in att if t[i, 1]], k)
    print("row workgroups")
    for k, name in ((0, "start"), (1, "qkv staged"), (2, "qkv arrived"), (3, "heads passed"), (4, "merged"),
                    (5, "end")):
        show(name, rows, k)
    m.close()


if __name__ == "__main__":
    main()
