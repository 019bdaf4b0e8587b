"""ctypes binding of the C ABI in include/xalm_hip.h (libxalm_hip.so, built in-tree).

There is no fallback: if the HIP library is missing or a call fails, this raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
# XALM_HIP_LIB: another build of the same library (launch-structure experiments, tools/)
HIP_LIB_PATH = os.environ.get("XALM_HIP_LIB") or os.path.join(LIB_DIR, "libxalm_hip.so")

# enum xh_dtype (the reference's Type ids, src/types.h:505-514)
F32, F16, BF16, F8_E4M3, F8_E5M2, U8, Q8 = 1, 2, 3, 6, 7, 8, 9
# the converter's gguf blocks (convert.py:176-187, quants.py): this build's ids
Q8_0, Q4_0 = 20, 21
DTYPE_BY_NAME = {"F32": F32, "F16": F16, "BF16": BF16, "F8_E4M3": F8_E4M3, "F8_E5M2": F8_E5M2,
                 "U8": U8, "Q8": Q8, "Q8_0": Q8_0, "Q4_0": Q4_0}
DTYPE_SIZE = {F32: 4, F16: 2, BF16: 2, F8_E4M3: 1, F8_E5M2: 1, U8: 1, Q8: 1}
GQ_BLOCK_BYTES = {Q8_0: 34, Q4_0: 18}  # bytes per 32-element block


def row_bytes(dtype: int, n: int) -> int:
    """Bytes of one n-element row as uploaded (gguf blocks: n/32 blocks)."""
    return n // 32 * GQ_BLOCK_BYTES[dtype] if dtype in GQ_BLOCK_BYTES else n * DTYPE_SIZE[dtype]
# enum xh_option
OPT_FUSE_ATTN_WO = 1
OPT_PREFILL = 2
OPT_PREFILL_GLU_SPLIT = 3
OPT_PREFILL_ATTN = 5
OPT_PREFILL_ATTN_SPLIT = 6

# enum xh_tensor_kind
EMBED, ATTN_NORM, FFN_NORM, WQ, WK, WV, WO, W1, W2, W3, FINAL_NORM, WCLS = range(12)
HYDRATE_KV_CACHE, OUTPUT_LOGITS = 0, 1
ACT_GELU, ACT_SILU = 0, 1


class XhConfig(ctypes.Structure):
    """POD mirror of `Config` (src/model.h:25-91)."""
    _fields_ = [("dim", ctypes.c_int32), ("hidden_dim", ctypes.c_int32), ("head_dim", ctypes.c_int32),
                ("n_layers", ctypes.c_int32), ("n_heads", ctypes.c_int32), ("n_kv_heads", ctypes.c_int32),
                ("vocab_size", ctypes.c_int32), ("max_seq_len", ctypes.c_int32), ("rope_theta", ctypes.c_float),
                ("rotary_dim", ctypes.c_int32), ("norm_eps", ctypes.c_float), ("act", ctypes.c_int32),
                ("qkv_clip", ctypes.c_float), ("tie_word_embeddings", ctypes.c_int32)]


class XhError(RuntimeError):
    pass


_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_SZ = ctypes.c_size_t
_FP = ctypes.POINTER(ctypes.c_float)

_SIGNATURES = {
    "xh_create": (_I, [ctypes.POINTER(XhConfig), _I, ctypes.POINTER(_P)]),
    "xh_destroy": (None, [_P]),
    "xh_last_error": (ctypes.c_char_p, [_P]),
    "xh_upload": (_I, [_P, _I, _I, _I, _P, _SZ]),
    "xh_upload_file": (_I, [_P, _I, _I, _I, ctypes.c_char_p, ctypes.c_uint64, _SZ]),
    "xh_upload_synthetic": (_I, [_P, _I, _I, _I, ctypes.c_uint64, ctypes.c_float, ctypes.c_float]),
    "xh_kv_fill_synthetic": (_I, [_P, _I, _I, _I, _I, ctypes.c_uint64, ctypes.c_float]),
    "xh_forward": (_I, [_P, _I, _I, _I, _P]),
    "xh_decode_greedy": (_I, [_P, _I, _I, _I, _I, _P, ctypes.POINTER(_I)]),
    "xh_prefill": (_I, [_P, _P, _I, _I, _I, _P]),
    "xh_perplexity": (_I, [_P, _P, _I, _I, _P]),
    "xh_debug_trace": (_I, [_P, _I, _P, _I, ctypes.POINTER(_I)]),
    "xh_get_logits": (_I, [_P, _P]),
    "xh_reset": (_I, [_P]),
    "xh_kv_write": (_I, [_P, _I, _I, _I, _I, _P]),
    "xh_kv_read": (_I, [_P, _I, _I, _I, _I, _P]),
    "xh_active_bytes": (_SZ, [_P, _SZ]),
    "xh_set_graphs": (_I, [_P, _I]),
    "xh_set_option": (_I, [_P, _I, _I]),
    "xh_get_option": (_I, [_P, _I, ctypes.POINTER(_I)]),
    "xh_op_matmul": (_I, [_P, _P, _P, _I, _I, _I]),
    "xh_op_rmsnorm": (_I, [_P, _P, _P, _I, _I, ctypes.c_float]),
    "xh_op_rope": (_I, [_P, _I, _I, _I, ctypes.c_float, _I]),
    "xh_op_mha": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I]),
    "xh_op_prompt_gemm": (_I, [_P, _P, _P, _P, _I, _I, _I, _I]),
    "xh_time_kernel": (_I, [_P, _I, _I, _FP]),
    "xh_kernel_bytes": (_SZ, [_P, _I, _I]),
}


def lib():
    """Load libxalm_hip.so (once).  Raises if it is absent: the product has no CPU fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(HIP_LIB_PATH):
            raise XhError(f"{HIP_LIB_PATH} not built (run `make` or __graft_entry__.build())")
        L = ctypes.CDLL(HIP_LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != 0:
        msg = lib().xh_last_error(ctx)
        raise XhError(f"xh error {rc}: {msg.decode() if msg else ''}")


def ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return ctypes.c_void_p(a.ctypes.data)


# ------------------------------------------------------------------------------------------
# op-level entry points (exposed-for-tests ops, src/model.h:286-316), numpy in / out
# ------------------------------------------------------------------------------------------
def op_matmul(x: np.ndarray, w: np.ndarray, dtype: int, n: int, d: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    w = np.ascontiguousarray(w)
    out = np.empty(d, dtype=np.float32)
    check(lib().xh_op_matmul(ptr(out), ptr(x), ptr(w), dtype, n, d))
    return out


def op_rmsnorm(x: np.ndarray, w: np.ndarray, dtype: int, eps: float) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    w = np.ascontiguousarray(w)
    out = np.empty_like(x)
    check(lib().xh_op_rmsnorm(ptr(out), ptr(x), ptr(w), dtype, x.size, eps))
    return out


def op_rope(vec: np.ndarray, head_dim: int, pos: int, theta: float, rotary_dim: int) -> np.ndarray:
    v = np.array(vec, dtype=np.float32, copy=True)
    check(lib().xh_op_rope(ptr(v), v.size, head_dim, pos, theta, rotary_dim))
    return v


def op_mha(kb: np.ndarray, vb: np.ndarray, q: np.ndarray, head_dim: int, kv_len: int, max_seq_len: int,
           n_heads: int, n_kv_heads: int) -> np.ndarray:
    kb = np.ascontiguousarray(kb, dtype=np.uint16)
    vb = np.ascontiguousarray(vb, dtype=np.uint16)
    q = np.ascontiguousarray(q, dtype=np.float32)
    out = np.empty(n_heads * head_dim, dtype=np.float32)
    check(lib().xh_op_mha(ptr(out), ptr(kb), ptr(vb), ptr(q), head_dim, kv_len, max_seq_len, n_heads, n_kv_heads))
    return out


def op_prompt_gemm(w: np.ndarray, xh: np.ndarray, xl: np.ndarray, ks: int = 0) -> np.ndarray:
    """The prompt-pass GEMM (gemm16.h): y[t][r] = sum_k w[r][k] (xh[t][k] + xl[t][k]); w, xh, xl
    f16 bit patterns (uint16) [rows][K], [n][K]; returns f32 [n][rows]."""
    w = np.ascontiguousarray(w, dtype=np.uint16)
    xh = np.ascontiguousarray(xh, dtype=np.uint16)
    xl = np.ascontiguousarray(xl, dtype=np.uint16)
    rows, K = w.shape
    n = xh.shape[0]
    assert xh.shape == (n, K) and xl.shape == (n, K)
    out = np.empty((n, rows), dtype=np.float32)
    check(lib().xh_op_prompt_gemm(ptr(out), ptr(w), ptr(xh), ptr(xl), rows, K, n, ks))
    return out
