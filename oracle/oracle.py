"""ctypes wrapper of the CPU oracle (liboracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "liboracle.so")

_P, _I, _SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-C", HERE], stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(LIB)
        sig = {
            "xo_create": (_P, [_P]), "xo_destroy": (None, [_P]),
            "xo_set_tensor": (_I, [_P, _I, _I, _I, _P]), "xo_forward": (_I, [_P, _I, _I, _I]),
            "xo_logits": (ctypes.POINTER(ctypes.c_float), [_P]),
            "xo_key_cache": (ctypes.POINTER(ctypes.c_uint16), [_P, _I]),
            "xo_value_cache": (ctypes.POINTER(ctypes.c_uint16), [_P, _I]),
            "xo_active_bytes": (_SZ, [_P, _SZ]), "xo_reset": (None, [_P]),
            "xo_matmul": (None, [_P, _P, _P, _I, _I, _I]),
            "xo_rmsnorm": (None, [_P, _P, _P, _I, _I, ctypes.c_float]),
            "xo_rope": (None, [_P, _I, _I, _I, ctypes.c_float, _I]),
            "xo_mha": (None, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I]),
            "xo_decode": (ctypes.c_float, [_I, _P, _SZ]),
            "xo_decode_row": (ctypes.c_float, [_I, _P, _SZ, _SZ, _SZ]),
            "xo_quantize_gq": (None, [_I, _P, _SZ, _P]),
            "xo_f32_to_f16": (ctypes.c_uint16, [ctypes.c_float]),
            "xo_f16_to_f32": (ctypes.c_float, [ctypes.c_uint16]),
            "xo_sample_argmax": (_I, [_P, _I]), "xo_sample_prob": (ctypes.c_float, [_P, _I, _I]),
            "xo_num_threads": (_I, []), "xo_set_threads": (None, [_I]),
            "xo_set_matmul_order": (None, [_I]), "xo_matmul_order": (_I, []), "xo_isa": (_I, []),
            "xo_fill_synthetic": (None, [_P, _SZ, _SZ, _I, ctypes.c_uint64, ctypes.c_float, ctypes.c_float]),
            "xo_set_precision": (None, [_P, _I]), "xo_precision": (_I, [_P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a):
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


class OracleModel:
    """Model::_forward_cpu restated in C (src/infer.cpp:604-638).  Borrows weight arrays."""

    def __init__(self, config):
        self.c = config
        self._keep = []
        self.m = _load().xo_create(ctypes.byref(config))
        if not self.m:
            raise MemoryError("xo_create failed")

    @classmethod
    def from_xalm(cls, xf, context=0):
        from xalm_amd import _lib as XL
        cfg = xf.config(context)
        m = cls(cfg)
        for kind, name in xf.global_tensors(bool(cfg.tie_word_embeddings)).items():
            m.set_tensor(kind, 0, xf.dtype(name), np.ascontiguousarray(xf.raw(name)))
        for layer in range(cfg.n_layers):
            for kind, name in xf.layer_tensors(layer).items():
                m.set_tensor(kind, layer, xf.dtype(name), np.ascontiguousarray(xf.raw(name)))
        _ = XL
        return m

    def set_tensor(self, kind, layer, dtype, arr):
        arr = np.ascontiguousarray(arr)
        self._keep.append(arr)
        rc = _load().xo_set_tensor(self.m, kind, layer, dtype, _p(arr))
        if rc:
            raise ValueError(f"xo_set_tensor rc={rc}")

    def set_precision(self, p):
        """1: this model's forward evaluated in double (every product, sum, norm, softmax,
        activation and residual), the fp16 K/V cache and the reference's float rope angles kept,
        logits rounded to float: the algorithm's value independent of f32 rounding order.
        0 (default): the reference's f32 arithmetic."""
        _load().xo_set_precision(self.m, int(p))

    def forward(self, token, pos, mode=1):
        rc = _load().xo_forward(self.m, int(token), int(pos), int(mode))
        if rc:
            raise RuntimeError(f"xo_forward rc={rc}")

    def logits(self):
        return np.ctypeslib.as_array(_load().xo_logits(self.m), shape=(self.c.vocab_size,)).copy()

    def kv(self, layer, which):
        kv_dim = self.c.n_kv_heads * self.c.head_dim
        fn = _load().xo_value_cache if which else _load().xo_key_cache
        return np.ctypeslib.as_array(fn(self.m, layer), shape=(self.c.max_seq_len, kv_dim)).copy()

    def set_kv(self, layer, which, slot0, rows):
        kv_dim = self.c.n_kv_heads * self.c.head_dim
        fn = _load().xo_value_cache if which else _load().xo_key_cache
        a = np.ctypeslib.as_array(fn(self.m, layer), shape=(self.c.max_seq_len, kv_dim))
        a[slot0: slot0 + rows.shape[0]] = rows

    def reset(self):
        _load().xo_reset(self.m)

    def active_bytes(self, pos):
        return int(_load().xo_active_bytes(self.m, pos))

    def close(self):
        if self.m:
            _load().xo_destroy(self.m)
            self.m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def matmul(x, w, dtype, n, d):
    x = np.ascontiguousarray(x, dtype=np.float32)
    w = np.ascontiguousarray(w)
    out = np.empty(d, dtype=np.float32)
    _load().xo_matmul(_p(out), _p(x), _p(w), dtype, n, d)
    return out


def rmsnorm(x, w, dtype, eps):
    x = np.ascontiguousarray(x, dtype=np.float32)
    w = np.ascontiguousarray(w)
    out = np.empty_like(x)
    _load().xo_rmsnorm(_p(out), _p(x), _p(w), dtype, x.size, eps)
    return out


def rope(vec, head_dim, pos, theta, rotary_dim):
    v = np.array(vec, dtype=np.float32, copy=True)
    _load().xo_rope(_p(v), v.size, head_dim, pos, theta, rotary_dim)
    return v


def mha(kb, vb, q, head_dim, kv_len, max_seq_len, n_heads, n_kv_heads):
    kb = np.ascontiguousarray(kb, dtype=np.uint16)
    vb = np.ascontiguousarray(vb, dtype=np.uint16)
    q = np.ascontiguousarray(q, dtype=np.float32)
    out = np.empty(n_heads * head_dim, dtype=np.float32)
    att = np.empty(n_heads * max_seq_len, dtype=np.float32)
    _load().xo_mha(_p(out), _p(att), _p(kb), _p(vb), _p(q), head_dim, kv_len, max_seq_len, n_heads, n_kv_heads)
    return out


def decode(dtype, arr, idx):
    arr = np.ascontiguousarray(arr)
    return float(_load().xo_decode(dtype, _p(arr), idx))


def f32_to_f16(f):
    return int(_load().xo_f32_to_f16(float(f)))


def f16_to_f32(h):
    return float(_load().xo_f16_to_f32(int(h)))


def sample_argmax(logits):
    logits = np.ascontiguousarray(logits, dtype=np.float32)
    return int(_load().xo_sample_argmax(_p(logits), logits.size))


def quantize_gq(dtype, values):
    """gguf Q8_0 / Q4_0 block bytes of float32 rows (len % 32 == 0), [rows][bytes]."""
    v = np.ascontiguousarray(values, dtype=np.float32)
    rows = v.shape[0] if v.ndim > 1 else 1
    nb = v.size // 32
    out = np.empty((rows, nb // rows * GQ_BLOCK_BYTES[dtype]), dtype=np.uint8)
    _load().xo_quantize_gq(dtype, _p(v), nb, _p(out))
    return out


def decode_row(dtype, data, row, n, i):
    data = np.ascontiguousarray(data)
    return float(_load().xo_decode_row(dtype, _p(data), row, n, i))


def sample_prob(logits, index):
    logits = np.ascontiguousarray(logits, dtype=np.float32)
    return float(_load().xo_sample_prob(_p(logits), logits.size, index))


def num_threads():
    return int(_load().xo_num_threads())


def set_threads(n):
    _load().xo_set_threads(int(n))


def set_matmul_order(order):
    """f16 / fp8 matmul in-row order: 0 = 8-wide FMA lanes (default), 1 = sequential.  Both read the
    reference's `omp simd` row loop (src/infer.cpp:104-135) validly; their difference is the
    reference algorithm's own rounding-order sensitivity."""
    _load().xo_set_matmul_order(int(order))


def isa():
    """the instruction set of the lanes-order matvec: 2 = AVX-512 (run-time dispatch), 1 = AVX2"""
    return int(_load().xo_isa())


def matmul_order():
    return int(_load().xo_matmul_order())


_NP = {1: np.float32, 2: np.uint16, 3: np.uint16, 6: np.uint8, 7: np.uint8, 20: np.uint8, 21: np.uint8}
GQ_BLOCK_BYTES = {20: 34, 21: 18}  # gguf Q8_0 / Q4_0: bytes per 32-element block


def synthetic(rows, cols, dtype, seed, mean, std):
    """Host copy of xh_upload_synthetic's tensor (include/xalm_synth.h), dense [rows][cols]
    (gguf blocks: [rows][cols/32 blocks] bytes, the converter's layout)."""
    if dtype in GQ_BLOCK_BYTES:
        out = np.empty((rows, cols // 32 * GQ_BLOCK_BYTES[dtype]), dtype=np.uint8)
        _load().xo_fill_synthetic(_p(out), rows, cols, dtype, seed, mean, std)
        return out
    out = np.empty((rows, cols) if rows > 1 else (cols,), dtype=_NP[dtype])
    _load().xo_fill_synthetic(_p(out), rows, cols, dtype, seed, mean, std)
    return out
