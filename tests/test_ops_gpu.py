"""Per-op parity: HIP kernels (through the C ABI) vs the CPU oracle on the same seeded inputs.

Ops are the reference's exposed-for-tests surface (src/model.h:286-316): matmul for every
weight dtype, rmsnorm, rope, multi-head attention (GQA, split-KV, long context).
Tolerances (fp32 accumulate, different summation order):
  matmul / attention : |gpu - cpu| <= 2e-6 * sum|terms| + 1e-7
  rmsnorm / rope     : |gpu - cpu| <= 4 ulp-scale (1e-6 relative)
"""
import numpy as np
import pytest

from oracle import oracle as O
from xalm_amd import _lib as L

pytestmark = pytest.mark.gpu


def rand_weights(rng, dtype, d, n, std=0.05):
    w = (rng.standard_normal((d, n)) * std).astype(np.float32)
    if dtype == L.F32:
        return w
    if dtype == L.F16:
        return w.astype(np.float16).view(np.uint16)
    if dtype == L.BF16:
        return (w.view(np.uint32) >> 16).astype(np.uint16)
    if dtype in (L.F8_E4M3, L.F8_E5M2, L.Q8):
        return rng.integers(0, 256, size=(d, n), dtype=np.uint8) if dtype != L.Q8 else \
            rng.integers(-128, 128, size=(d, n), dtype=np.int8)
    raise ValueError(dtype)


def decoded(w, dtype):
    flat = np.ascontiguousarray(w).reshape(-1)
    if dtype == L.F32:
        return flat.view(np.float32).astype(np.float64)
    if dtype == L.F16:
        return flat.view(np.float16).astype(np.float64)
    if dtype == L.BF16:
        return (flat.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    # one-byte codes: the oracle's decode of each of the 256 codes, gathered by code
    codes = np.arange(256, dtype=np.uint8)
    table = np.array([O.decode(dtype, codes.view(np.int8) if dtype == L.Q8 else codes, i) for i in range(256)],
                     dtype=np.float64)
    return table[flat.view(np.uint8)]


@pytest.mark.parametrize("dtype", [L.F16, L.BF16, L.F32, L.F8_E4M3, L.F8_E5M2, L.Q8])
@pytest.mark.parametrize("n,d", [(64, 32), (512, 96), (4096, 64), (1536, 300), (14336, 8)])
def test_matmul(dtype, n, d):
    rng = np.random.default_rng(n * 7 + d + dtype)
    x = rng.standard_normal(n).astype(np.float32)
    w = rand_weights(rng, dtype, d, n)
    got = L.op_matmul(x, w, dtype, n, d)
    cpu = O.matmul(x, w, dtype, n, d)
    wd = decoded(w, dtype).reshape(d, n)
    mag = np.abs(wd) @ np.abs(x.astype(np.float64))
    assert np.all(np.abs(got - cpu) <= 2e-6 * mag + 1e-7), np.abs(got - cpu).max()


@pytest.mark.parametrize("dtype", [L.BF16, L.F32])
@pytest.mark.parametrize("n", [64, 512, 4096, 14336])
def test_rmsnorm(dtype, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32) * 3
    wf = (1 + 0.1 * rng.standard_normal(n)).astype(np.float32)
    w = wf if dtype == L.F32 else (wf.view(np.uint32) >> 16).astype(np.uint16)
    got = L.op_rmsnorm(x, w, dtype, 1e-5)
    cpu = O.rmsnorm(x, w, dtype, 1e-5)
    assert np.allclose(got, cpu, rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("pos", [0, 1, 7, 4095, 32767, 100000])
@pytest.mark.parametrize("head_dim,rot", [(128, 128), (16, 16), (64, 32)])
def test_rope(pos, head_dim, rot):
    rng = np.random.default_rng(pos + head_dim)
    v = rng.standard_normal(4 * head_dim).astype(np.float32)
    got = L.op_rope(v, head_dim, pos, 1e6, rot)
    cpu = O.rope(v, head_dim, pos, 1e6, rot)
    # device cosf/sinf (ocml) vs host libm: <= ~2 ulp of the rotated value's magnitude
    assert np.abs(got - cpu).max() <= 2e-6 * np.abs(v).max() * 2, np.abs(got - cpu).max()


def f16(a):
    return a.astype(np.float16).view(np.uint16)


# (256, 16, 2): 8 q heads per KV head x 256 = 2048 outputs per block, more than its 1024 threads
# (the last split's merge covers them in rounds)
@pytest.mark.parametrize("head_dim,n_heads,n_kv", [(128, 32, 8), (128, 4, 1), (16, 4, 2), (64, 8, 8), (32, 8, 1),
                                                   (256, 16, 2)])
@pytest.mark.parametrize("kv_len,msl", [(1, 64), (17, 64), (300, 4096), (4096, 4096), (100, 128)])
def test_mha(head_dim, n_heads, n_kv, kv_len, msl):
    rng = np.random.default_rng(kv_len * 131 + head_dim + n_heads)
    kv_dim = n_kv * head_dim
    kb = f16(rng.standard_normal((msl, kv_dim)).astype(np.float32))
    vb = f16(rng.standard_normal((msl, kv_dim)).astype(np.float32))
    q = (rng.standard_normal(n_heads * head_dim) * 0.5).astype(np.float32)
    got = L.op_mha(kb, vb, q, head_dim, kv_len, msl, n_heads, n_kv)
    cpu = O.mha(kb, vb, q, head_dim, kv_len, msl, n_heads, n_kv)
    # outputs are convex combinations of V rows (|v| ~ 1..4): absolute bound
    assert np.abs(got - cpu).max() < 2e-5, np.abs(got - cpu).max()


@pytest.mark.parametrize("n_heads,n_kv", [(32, 8), (8, 8), (16, 8)])
@pytest.mark.parametrize("kv_len", [257, 1000, 8191, 20001])
def test_mha_long_splits(n_heads, n_kv, kv_len):
    """Splits of 256..1024 slots at head_dim 128 with 4, 1 and 2 q heads per KV head (ragged
    last rounds, many partials merged by the last split) against the oracle's per-head loop."""
    rng = np.random.default_rng(kv_len + 7 * n_heads)
    head_dim, msl = 128, 32768
    kv_dim = n_kv * head_dim
    kb = f16(rng.standard_normal((msl, kv_dim)).astype(np.float32))
    vb = f16(rng.standard_normal((msl, kv_dim)).astype(np.float32))
    q = (rng.standard_normal(n_heads * head_dim) * 0.5).astype(np.float32)
    got = L.op_mha(kb, vb, q, head_dim, kv_len, msl, n_heads, n_kv)
    cpu = O.mha(kb, vb, q, head_dim, kv_len, msl, n_heads, n_kv)
    assert np.abs(got - cpu).max() < 2e-5, np.abs(got - cpu).max()


def test_mha_peaked_softmax_and_32k():
    # one key dominates (forces the split max-rescale path), long context split over many blocks
    rng = np.random.default_rng(5)
    head_dim, n_heads, n_kv, msl, kv_len = 128, 32, 8, 32768, 32768
    kv_dim = n_kv * head_dim
    kb = f16((rng.standard_normal((msl, kv_dim)) * 0.3).astype(np.float32))
    vb = f16(rng.standard_normal((msl, kv_dim)).astype(np.float32))
    q = rng.standard_normal(n_heads * head_dim).astype(np.float32)
    spike = 20000
    kb[spike] = f16(np.tile(q[:head_dim] / np.linalg.norm(q[:head_dim]) * 8, n_kv).astype(np.float32))
    got = L.op_mha(kb, vb, q, head_dim, kv_len, msl, n_heads, n_kv)
    cpu = O.mha(kb, vb, q, head_dim, kv_len, msl, n_heads, n_kv)
    assert np.abs(got - cpu).max() < 5e-5, np.abs(got - cpu).max()


def _special(codes, dtype):
    # OCP NaN/Inf patterns, where gfx950's converter and the reference's bit decode differ
    return (codes & 0x7C) == 0x7C if dtype == L.F8_E5M2 else (codes & 0x7F) == 0x7F


@pytest.mark.parametrize("dtype", [L.F8_E4M3, L.F8_E5M2])
@pytest.mark.parametrize("with_special", [False, True])
def test_f8_decode_every_code(dtype, with_special):
    """Every fp8 code through the matvec, bit-exact against the reference decode
    (src/types.h:302-314).  Without NaN/Inf codes the matrix takes the hardware converter
    (v_cvt_pk_f32_fp8/_bf8); with them, the exact bit form."""
    codes = np.arange(256, dtype=np.uint8)
    if not with_special:
        codes = codes[~_special(codes, dtype)]
    d, n = codes.size, 64
    w = np.zeros((d, n), dtype=np.uint8)
    w[:, 5] = codes  # one nonzero column: y[r] = decode(code r) * 1.0, exactly
    x = np.zeros(n, dtype=np.float32)
    x[5] = 1.0
    got = L.op_matmul(x, w, dtype, n, d)
    ref = np.array([O.decode(dtype, codes, i) for i in range(d)], dtype=np.float32)
    ref = ref + np.float32(0.0)  # the fp32 sum starts at +0: code 0x80 (-0) sums to +0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("dtype", [L.F8_E4M3, L.F8_E5M2])
@pytest.mark.parametrize("n,d", [(4096, 64), (1536, 96)])
def test_matmul_f8_hw(dtype, n, d):
    """Random finite fp8 weights (the converter path) vs the oracle."""
    rng = np.random.default_rng(n + d + dtype)
    x = rng.standard_normal(n).astype(np.float32)
    w = rng.integers(0, 256, size=(d, n), dtype=np.uint8)
    w[_special(w, dtype)] = 0x01
    got = L.op_matmul(x, w, dtype, n, d)
    cpu = O.matmul(x, w, dtype, n, d)
    wd = decoded(w, dtype).reshape(d, n)
    mag = np.abs(wd) @ np.abs(x.astype(np.float64))
    assert np.all(np.abs(got - cpu) <= 2e-6 * mag + 1e-7), np.abs(got - cpu).max()


def split16(x):
    """prefill_split_kernel's exact f16 hi + lo of rows scaled into [2^14, 2^15) (float64 ref)"""
    m = np.abs(x).max(axis=1, keepdims=True)
    s = np.exp2(15 - np.ceil(np.log2(np.where(m > 0, m, 1.0)) + 1e-12))
    u = (x * s).astype(np.float32)
    hi = u.astype(np.float16)
    lo = (u - hi.astype(np.float32)).astype(np.float16)
    return hi.view(np.uint16), lo.view(np.uint16)


@pytest.mark.parametrize("rows,K,n,ks", [(256, 64, 1, 1), (300, 128, 37, 0), (1000, 512, 200, 4), (6144, 4096, 512, 0),
                                         (4096, 14336, 130, 0), (28672, 4096, 64, 2), (512, 4096, 1100, 1),
                                         (4096, 4096, 1024, 8)])
def test_prompt_gemm(rows, K, n, ks):
    """The prompt-pass GEMM (gemm16.h) vs a float64 sum of the same f16 products: ragged row and
    token tiles (clamped loads), 1 to 8 K slices, Mistral-7B shapes; |err| <= 1e-5 sum|terms|
    (f32 accumulation over up to 14336 products), and bitwise equal on a second launch."""
    rng = np.random.default_rng(rows + K + n)
    w = (rng.standard_normal((rows, K)) * 0.02).astype(np.float16)
    x = rng.standard_normal((n, K))
    xh, xl = split16(x)
    got = L.op_prompt_gemm(w.view(np.uint16), xh, xl, ks)
    assert got.shape == (n, rows)
    assert np.array_equal(got.view(np.uint32), L.op_prompt_gemm(w.view(np.uint16), xh, xl, ks).view(np.uint32))
    sel = rng.choice(rows, size=min(rows, 96), replace=False)
    wd = w[sel].astype(np.float64)
    xd = xh.view(np.float16).astype(np.float64) + xl.view(np.float16).astype(np.float64)
    ref = xd @ wd.T
    mag = np.abs(xd) @ np.abs(wd).T
    err = np.abs(got[:, sel] - ref)
    assert np.all(err <= 1e-5 * mag + 1e-7), float((err / (mag + 1e-30)).max())


def test_prompt_gemm_rejects_bad_shapes():
    w = np.zeros((64, 96), np.uint16)
    x = np.zeros((4, 96), np.uint16)
    with pytest.raises(L.XhError):
        L.op_prompt_gemm(w, x, x)  # K not a multiple of 64
    w = np.zeros((64, 128), np.uint16)
    x = np.zeros((4, 128), np.uint16)
    with pytest.raises(L.XhError):
        L.op_prompt_gemm(w, x, x, 4)  # 4 slices of 32
