"""Timeline of one fused W1/W3 + W2 launch (mlp.h; the last layer of the last decoded token)."""
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
    args = ap.parse_args()
    w = bench.WORKLOADS[args.workload]
    c = bench.make_config(w)
    m = Model(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        m.upload_synthetic(kind, layer, dt, seed, mean, std)
    m.set_option(L.OPT_FUSE_MLP, 1)
    st = InferenceState(c)
    prompt = bench.prompt_tokens(c.vocab_size)
    m.prefill(prompt, 0, st)
    m.decode_greedy(len(prompt), 100)
    m.debug_trace(4)
    m.decode_greedy(len(prompt) + 100, 2)
    tr = m.debug_trace(0).astype(np.int64)
    t = tr[: tr.size // 4 * 4].reshape(-1, 4)
    used = np.nonzero(t[:, 0])[0]
    t0 = t[used, 0].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731
    nb13 = 256  # MLP_WAVES / 8 waves per workgroup (W1/W3 groups divide evenly at these shapes)
    for name, blocks in (("w1/w3", [i for i in used if i < nb13]), ("w2", [i for i in used if i >= nb13])):
        print(f"{name}: {len(blocks)} workgroups")
        for k, lab in ((0, "start"), (1, "rows done" if name == "w1/w3" else "hb ready"), (2, "end")):
            v = np.array([us(t[i, k]) for i in blocks if t[i, k]])
            if v.size:
                q = np.percentile(v, [10, 50, 90])
                print(f"  {lab:10s} min {v.min():7.2f} p10 {q[0]:7.2f} med {q[1]:7.2f} p90 {q[2]:7.2f} max {v.max():7.2f} us")
    m.close()


if __name__ == "__main__":
    main()
