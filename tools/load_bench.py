"""Weight-load throughput: xh_upload_file (mmap + MAP_POPULATE -> registered -> one DMA) vs the host path
(np.memmap -> xh_upload: a pageable copy from the mapping; the reference reads into a host Tensor).

Writes a scratch file holding `--layers` Mistral-7B W1/W3 pairs (f16, 224 MiB per layer)
and loads them into one device context both ways.  The first pass over the file also pages
it into the host page cache, so both timed paths read from cache: this measures the
loader's host->HBM rate, not the disk.

    python tools/load_bench.py --layers 8 --dir /tmp
"""
import argparse
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import Model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--dir", default=tempfile.gettempdir())
    args = ap.parse_args()
    cfg = L.XhConfig()
    cfg.dim, cfg.hidden_dim, cfg.head_dim, cfg.n_layers = 4096, 14336, 128, args.layers
    cfg.n_heads, cfg.n_kv_heads, cfg.vocab_size, cfg.max_seq_len = 32, 8, 512, 64
    cfg.rope_theta, cfg.rotary_dim, cfg.norm_eps, cfg.act = 1e6, 128, 1e-5, L.ACT_SILU
    cfg.qkv_clip, cfg.tie_word_embeddings = float(np.finfo(np.float32).max), 0
    nbytes = 14336 * 4096 * 2
    path = os.path.join(args.dir, f"load_bench_{os.getpid()}.bin")
    block = np.random.default_rng(0).integers(0, 1 << 15, nbytes // 2, dtype=np.uint16).tobytes()
    try:
        with open(path, "wb") as f:
            for _ in range(2 * args.layers):
                f.write(block)
        mm = np.memmap(path, dtype=np.uint8, mode="r")
        total = 2 * args.layers * nbytes
        res = {}
        for name in ("warm", "file", "host"):
            gm = Model(cfg)
            t0 = time.perf_counter()
            for layer in range(args.layers):
                for j, kind in enumerate((L.W1, L.W3)):
                    off = (2 * layer + j) * nbytes
                    if name == "host":
                        gm.upload(kind, layer, L.F16, np.ascontiguousarray(mm[off: off + nbytes]))
                    else:
                        gm.upload_file(kind, layer, L.F16, path, off, nbytes)
            dt = time.perf_counter() - t0
            gm.close()
            res[name] = total / dt / 1e9
            print(f"{name:5s} {total / 2**30:.2f} GiB in {dt * 1e3:.1f} ms = {res[name]:.2f} GB/s", flush=True)
        print(f"xh_upload_file / host path: {res['file'] / res['host']:.2f}x")
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
