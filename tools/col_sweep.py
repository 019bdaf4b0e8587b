"""Column-form attention + Wo (attn_col.h) vs the split form, per history length, Mistral-7B
shapes: xh_time_kernel 6 (column form), 5 (split attention alone), 2 (Wo matvec alone)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402

w = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "mistral-7b-f16"]
c = bench.make_config(w)
m = Model(c)
for kind, layer, dt, seed, mean, std in bench.tensor_specs(w):
    m.upload_synthetic(kind, layer, dt, seed, mean, std)
m.set_option(L.OPT_COL_KV_MAX, 256)
st = InferenceState(c)
for kv in (1, 16, 64, 128, 129, 200, 256):
    m.forward(st, 5, kv - 1, L.HYDRATE_KV_CACHE)
    r = {}
    for which, name in ((6, "col"), (5, "attn"), (2, "wo"), (7, "w13p"), (0, "w13")):
        r[name] = m.time_kernel(which, 100)
    print(f"kv {kv:5d}: " + "  ".join(f"{k} {v:6.2f}" for k, v in r.items()), flush=True)
m.close()
