"""Timeline of one fused attention + Wo launch (the last layer of the last decoded token)."""
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
    ap.add_argument("--fuse", type=int, default=1, help="XH_OPT_FUSE_ATTN_WO (2: W1/W3 role traced too)")
    ap.add_argument("--aw-threads", type=int, default=1024, help="AW_THREADS of the library (XALM_HIP_LIB)")
    ap.add_argument("--pos0", type=int, default=0, help="4k workloads: synthetic K/V history [0, pos0) first "
                    "(e.g. 3800: the traced token attends over ~4k slots)")
    args = ap.parse_args()
    w = bench.WORKLOADS[args.workload]
    c = bench.make_config(w)
    m = Model(c)
    for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
        m.upload_synthetic(kind, layer, dt, seed, mean, std)
    from xalm_amd import _lib as L
    m.set_option(L.OPT_FUSE_ATTN_WO, args.fuse)
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
        for layer in range(c.n_layers if args.pos0 else 0):
            m.kv_fill_synthetic(layer, 0, 0, args.pos0, 5000 + 2 * layer, 1.0)
            m.kv_fill_synthetic(layer, 1, 0, args.pos0, 5001 + 2 * layer, 1.0)
        m.prefill(prompt, args.pos0, st)
        m.decode_greedy(args.pos0 + len(prompt), 200)
        pos = args.pos0 + len(prompt) + 200
    m.debug_trace(2)
    m.decode_greedy(pos, 2)
    tr = m.debug_trace(0).astype(np.int64)
    nkv = c.n_kv_heads
    n = tr.size // 8
    t = tr[: n * 8].reshape(n, 8)
    used = np.nonzero(t[:, 0])[0]
    t0 = t[used, 0].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731
    nsplit = None
    # attention workgroups: stamp 1 = done (0 if it exited as an inactive split: then = start)
    nsplit = max(1, min(256 // nkv, 128, (c.max_seq_len + 255) // 256))  # attn_nsplit (xalm_hip.hip)
    # Wo workgroups (AwShape: 16 waves x 2 rows, one round of <= 4096 waves): ceil(dim / 32)
    rows_per_wg = 2 * args.aw_threads // 64
    nb_wo = (c.dim + rows_per_wg - 1) // rows_per_wg
    att = [i for i in used if i < nkv * nsplit]
    wo = [i for i in used if nkv * nsplit <= i < nkv * nsplit + nb_wo]
    mlp = [i for i in used if i >= nkv * nsplit + nb_wo]
    print(f"workgroups traced: {len(used)} (attention {len(att)}, wo {len(wo)}, w1/w3 {len(mlp)})")
    if att:
        a_start = np.array([us(t[i, 0]) for i in att])
        a_done = np.array([us(t[i, 1]) for i in att if t[i, 1]])
        print(f"attention start  min {a_start.min():6.2f} max {a_start.max():6.2f} us")
        if a_done.size:
            print(f"attention done   min {a_done.min():6.2f} med {np.median(a_done):6.2f} max {a_done.max():6.2f} us")
        if a_done.size:
            per = []
            for g in range(nkv):
                d = [us(t[i, 1]) for i in att if i // nsplit == g and t[i, 1]]
                if d:
                    per.append(f"h{g} {np.median(d):5.1f}/{max(d):5.1f}")
            print("  done per KV head (median/max us): " + "  ".join(per))
        act = [i for i in att if t[i, 5]]
        for k, name in ((2, "split known"), (3, "scores done"), (6, "softmax done"), (7, "p.V summed"), (4, "p.V reduced"),
                        (5, "partial drained"), (1, "signalled")):
            v = np.array([us(t[i, k]) for i in act])
            if v.size:
                print(f"  {name:15s} min {v.min():6.2f} med {np.median(v):6.2f} max {v.max():6.2f} us")
    if wo:
        for k, name in ((0, "wo start"), (1, "wo passed"), (3, "wo staged"), (2, "wo end"), (4, "wo x published")):
            v = np.array([us(t[i, k]) for i in wo if t[i, k]])
            if v.size:
                print(f"{name:15s}  min {v.min():6.2f} med {np.median(v):6.2f} max {v.max():6.2f} us")
    if mlp:
        for k, name in ((0, "w13 start"), (1, "w13 x ready"), (2, "w13 end")):
            v = np.array([us(t[i, k]) for i in mlp if t[i, k]])
            if v.size:
                q = np.percentile(v, [10, 50, 90])
                print(f"{name:15s}  min {v.min():6.2f} p10 {q[0]:6.2f} med {q[1]:6.2f} p90 {q[2]:6.2f} max {v.max():6.2f} us")
        st_ = np.array(sorted(us(t[i, 0]) for i in mlp))
        print("w13 workgroups started by 2/5/10/15/20/30 us:",
              [int((st_ <= x).sum()) for x in (2, 5, 10, 15, 20, 30)], "of", len(mlp))
    m.close()


if __name__ == "__main__":
    main()
