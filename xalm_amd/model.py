"""Host-side mirror of the reference `Model` / `InferenceState` API over the C ABI.

    model = Model.from_xalm(XalmFile(path), context=0, device=0)   # src/model.cpp:48-118
    state = InferenceState(model.config)                             # src/model.h:96-156
    model.forward(state, token, pos, mode=OUTPUT_LOGITS)             # src/model.h:272
    state.logits()                                                   # host float[vocab]

Every call goes to libxalm_hip.so (HIP kernels on gfx950); errors raise XhError, as the
reference loader throws.  There is no CPU path here.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L
from .xalm_file import XalmFile


class InferenceState:
    """Host view of the device state: only `logits` crosses back."""

    def __init__(self, config: L.XhConfig):
        self._logits = np.zeros(config.vocab_size, dtype=np.float32)

    def logits(self) -> np.ndarray:
        return self._logits


class Model:
    def __init__(self, config: L.XhConfig, device: int = 0):
        self.config = config
        self._ctx = ctypes.c_void_p()
        L.check(L.lib().xh_create(ctypes.byref(config), device, ctypes.byref(self._ctx)))

    # -- construction ----------------------------------------------------------------
    @classmethod
    def from_xalm(cls, xf: XalmFile, context: int = 0, device: int = 0, direct: bool = True) -> "Model":
        """`direct`: tensors stream from the file into device memory (xh_upload_file);
        otherwise each one is read on the host and copied (xh_upload)."""
        cfg = xf.config(context)
        m = cls(cfg, device)
        c = cfg
        shapes = {L.EMBED: (c.vocab_size, c.dim), L.FINAL_NORM: (c.dim,), L.WCLS: (c.vocab_size, c.dim)}
        for kind, name in xf.global_tensors(bool(c.tie_word_embeddings)).items():
            m._load(xf, kind, 0, name, shapes[kind], direct)
        q_dim, kv_dim = c.n_heads * c.head_dim, c.n_kv_heads * c.head_dim
        lshapes = {L.ATTN_NORM: (c.dim,), L.FFN_NORM: (c.dim,), L.WQ: (q_dim, c.dim), L.WK: (kv_dim, c.dim),
                   L.WV: (kv_dim, c.dim), L.WO: (c.dim, q_dim), L.W1: (c.hidden_dim, c.dim),
                   L.W2: (c.dim, c.hidden_dim), L.W3: (c.hidden_dim, c.dim)}
        for layer in range(c.n_layers):
            for kind, name in xf.layer_tensors(layer).items():
                m._load(xf, kind, layer, name, lshapes[kind], direct)
        return m

    def _load(self, xf: XalmFile, kind: int, layer: int, name: str, expected_shape, direct: bool = True):
        ti = xf.tensors[name]
        dt = xf.dtype(name)
        if dt in L.GQ_BLOCK_BYTES and len(expected_shape) == 2 and expected_shape[1] % 32 == 0:
            # gguf blocks (convert.py:176-187): the header holds the byte shape
            expected_shape = (expected_shape[0], expected_shape[1] // 32 * L.GQ_BLOCK_BYTES[dt])
        if tuple(ti.shape) != tuple(expected_shape):  # src/model.cpp:65-76
            raise ValueError(f"shape mismatch for {name}: {ti.shape} vs {expected_shape} expected!")
        if direct:
            self.upload_file(kind, layer, xf.dtype(name), xf.path, ti.offset, ti.size)
        else:
            self.upload(kind, layer, xf.dtype(name), np.ascontiguousarray(xf.raw(name)))

    def upload(self, kind: int, layer: int, dtype: int, data: np.ndarray):
        data = np.ascontiguousarray(data)
        L.check(L.lib().xh_upload(self._ctx, kind, layer, dtype, L.ptr(data), data.nbytes), self._ctx)

    def upload_file(self, kind: int, layer: int, dtype: int, path: str, offset: int, nbytes: int):
        L.check(L.lib().xh_upload_file(self._ctx, kind, layer, dtype, str(path).encode(), int(offset), int(nbytes)),
                self._ctx)

    def upload_synthetic(self, kind: int, layer: int, dtype: int, seed: int, mean: float, std: float):
        L.check(L.lib().xh_upload_synthetic(self._ctx, kind, layer, dtype, seed, mean, std), self._ctx)

    def kv_fill_synthetic(self, layer: int, which: int, slot0: int, n_slots: int, seed: int, std: float):
        L.check(L.lib().xh_kv_fill_synthetic(self._ctx, layer, which, slot0, n_slots, seed, std), self._ctx)

    # -- inference -----------------------------------------------------------------------
    def forward(self, s: InferenceState, token: int, pos: int, mode: int = L.OUTPUT_LOGITS):
        out = L.ptr(s.logits()) if mode == L.OUTPUT_LOGITS else None
        L.check(L.lib().xh_forward(self._ctx, int(token), int(pos), int(mode), out), self._ctx)

    def decode_greedy(self, pos: int, n_steps: int, stop=(-1, -1)) -> list[int]:
        toks = np.zeros(max(n_steps, 1), dtype=np.int32)
        done = ctypes.c_int(0)
        L.check(L.lib().xh_decode_greedy(self._ctx, int(pos), int(n_steps), int(stop[0]), int(stop[1]),
                                         L.ptr(toks), ctypes.byref(done)), self._ctx)
        return toks[: done.value].tolist()

    def prefill(self, tokens, pos0: int, s: InferenceState | None = None) -> None:
        """Hydrate tokens[0..n) at positions pos0.. (the prompt loop of run_completion,
        src/main.cpp:94-100); the last token's logits land in `s` when given."""
        toks = np.ascontiguousarray(np.asarray(tokens, dtype=np.int32))
        out = L.ptr(s.logits()) if s is not None else None
        L.check(L.lib().xh_prefill(self._ctx, L.ptr(toks), int(toks.size), int(pos0), int(s is not None), out),
                self._ctx)

    def token_probs(self, tokens, pos0: int = 0) -> np.ndarray:
        """run_perplexity's loop (src/main.cpp:243-254) on the device: forward tokens[:-1] at
        positions pos0.., element i = Sampler::sample_prob(tokens[i + 1]) after token i."""
        toks = np.ascontiguousarray(np.asarray(tokens, dtype=np.int32))
        out = np.zeros(max(toks.size - 1, 1), dtype=np.float32)
        L.check(L.lib().xh_perplexity(self._ctx, L.ptr(toks), int(toks.size), int(pos0), L.ptr(out)), self._ctx)
        return out[: toks.size - 1]

    def debug_trace(self, enable: int = -1) -> np.ndarray:
        """Timeline of the last traced attention + Wo launch, [workgroup][8] device-clock stamps
        (100 MHz, attn_wo.h); `enable` 2/0 switches tracing for later launches."""
        n = ctypes.c_int(0)
        L.check(L.lib().xh_debug_trace(self._ctx, -1, None, 0, ctypes.byref(n)), self._ctx)
        out = np.zeros(n.value, dtype=np.uint64)
        L.check(L.lib().xh_debug_trace(self._ctx, int(enable), L.ptr(out), n.value, ctypes.byref(n)), self._ctx)
        return out

    def get_logits(self, s: InferenceState):
        L.check(L.lib().xh_get_logits(self._ctx, L.ptr(s.logits())), self._ctx)

    def reset(self):
        L.check(L.lib().xh_reset(self._ctx), self._ctx)

    def set_graphs(self, enable: bool):
        L.check(L.lib().xh_set_graphs(self._ctx, int(enable)), self._ctx)

    def set_option(self, option: int, value: int):
        L.check(L.lib().xh_set_option(self._ctx, int(option), int(value)), self._ctx)

    def get_option(self, option: int) -> int:
        v = ctypes.c_int(0)
        L.check(L.lib().xh_get_option(self._ctx, int(option), ctypes.byref(v)), self._ctx)
        return int(v.value)

    def active_bytes(self, pos: int) -> int:
        return int(L.lib().xh_active_bytes(self._ctx, pos))

    def kv_write(self, layer: int, which: int, slot0: int, rows: np.ndarray):
        rows = np.ascontiguousarray(rows, dtype=np.uint16)
        n = rows.shape[0]
        L.check(L.lib().xh_kv_write(self._ctx, layer, which, slot0, n, L.ptr(rows)), self._ctx)

    def kv_read(self, layer: int, which: int, slot0: int, n_slots: int) -> np.ndarray:
        kv_dim = self.config.n_kv_heads * self.config.head_dim
        out = np.empty((n_slots, kv_dim), dtype=np.uint16)
        L.check(L.lib().xh_kv_read(self._ctx, layer, which, slot0, n_slots, L.ptr(out)), self._ctx)
        return out

    def time_kernel(self, which: int, iters: int) -> float:
        us = ctypes.c_float(0)
        L.check(L.lib().xh_time_kernel(self._ctx, which, iters, ctypes.byref(us)), self._ctx)
        return float(us.value)

    def kernel_bytes(self, which: int, kv_len: int) -> int:
        return int(L.lib().xh_kernel_bytes(self._ctx, which, kv_len))

    def close(self):
        if self._ctx:
            L.lib().xh_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
