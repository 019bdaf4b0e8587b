"""Per-workgroup finish times of one plain W1/W3 launch (the last layer of the last decoded token):
how unevenly the HBM stream serves the CUs (gemv.h trace: start, x staged, end, XCD / HW_ID)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
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
    st = InferenceState(c)
    prompt = bench.prompt_tokens(c.vocab_size)
    m.prefill(prompt, 0, st)
    m.decode_greedy(len(prompt), 50)
    m.debug_trace(8)
    m.decode_greedy(len(prompt) + 50, 2)
    tr = m.debug_trace(0)
    t = tr[: tr.size // 4 * 4].reshape(-1, 4)
    used = np.nonzero(t[:, 0])[0]
    t = t[used]
    t0 = t[:, 0].min()
    st_, sg, en = [(t[:, k].astype(np.int64) - t0) / 100.0 for k in (0, 1, 2)]
    xcc = (t[:, 3] >> 32).astype(np.int64)
    hw = (t[:, 3] & 0xFFFFFFFF).astype(np.int64)
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    print(f"{len(used)} workgroups; start max {st_.max():.2f}  staged med {np.median(sg):.2f}  end min {en.min():.2f} "
          f"p10 {np.percentile(en, 10):.2f} med {np.median(en):.2f} p90 {np.percentile(en, 90):.2f} max {en.max():.2f} us")
    for k in range(8):
        e = en[xcc == k]
        if e.size:
            print(f"  XCD {k}: {e.size:3d} wgs  end min {e.min():6.2f} med {np.median(e):6.2f} max {e.max():6.2f}")
    # per CU (XCD, SE, SH, CU): workgroups per CU and their end times
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    uk, cnt = np.unique(key, return_counts=True)
    print("workgroups per CU:", dict(zip(*np.unique(cnt, return_counts=True))))
    ends = {k: en[key == k].max() for k in uk}
    two = [ends[k] for k, c_ in zip(uk, cnt) if c_ == 2]
    one = [ends[k] for k, c_ in zip(uk, cnt) if c_ == 1]
    if two:
        print(f"  CUs with 2 wgs: end med {np.median(two):.2f} max {max(two):.2f}")
    if one:
        print(f"  CUs with 1 wg : end med {np.median(one):.2f} max {max(one):.2f}")
    hist = np.histogram(en, bins=10)
    print("end histogram:", [int(x) for x in hist[0]], "edges", [round(float(x), 1) for x in hist[1]])
    m.close()


if __name__ == "__main__":
    main()
