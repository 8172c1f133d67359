"""Kernel-level parity of the HIP path (through the C ABI) against the CPU oracle /
a plain fp32 reference of the same op.  Tolerances are stated per test."""
import ctypes as C

import numpy as np
import pytest

from oracle import dtw as odtw
from oracle import mel as omel
from wdr import _lib
import wdr

pytestmark = pytest.mark.gpu

U16 = C.POINTER(C.c_uint16)
F32 = C.POINTER(C.c_float)
I32 = C.POINTER(C.c_int32)


def _f16bits(a):
    return np.ascontiguousarray(a.astype(np.float16)).view(np.uint16)


def _proj(lib, a, w, bias, epi, out0=None):
    M, K = a.shape
    N = w.shape[0]
    out = np.zeros((M, N), np.float32) if out0 is None else out0.copy()
    ab, wb = _f16bits(a), _f16bits(w)
    b = None if bias is None else np.ascontiguousarray(bias, np.float32)
    _lib.check(lib.wdr_dbg_proj(ab.ctypes.data_as(U16), wb.ctypes.data_as(U16),
                                None if b is None else b.ctypes.data_as(F32), M, N, K, epi, out.ctypes.data_as(F32)))
    return out


def _gelu(x):
    return 0.5 * x * (1 + np.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


@pytest.mark.parametrize("M", [1, 3, 8, 9, 17, 33, 64, 65, 300, 1500])
def test_projection_matches_fp32_reference(lib, M):
    rng = np.random.default_rng(M)
    K, N = 256, 384
    a = rng.standard_normal((M, K)).astype(np.float16).astype(np.float32)
    w = (rng.standard_normal((N, K)) * 0.05).astype(np.float16).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    ref = a.astype(np.float64) @ w.T.astype(np.float64) + bias
    # f32 output: accumulation-order error only
    np.testing.assert_allclose(_proj(lib, a, w, bias, 3), ref, rtol=0, atol=2e-4)
    # f16 output (+GELU): f16 rounding of the result, |err| <= 2^-10 relative
    np.testing.assert_allclose(_proj(lib, a, w, bias, 0), ref, rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(_proj(lib, a, w, bias, 1), _gelu(ref), rtol=2e-3, atol=2e-3)
    base = rng.standard_normal((M, N)).astype(np.float32)
    np.testing.assert_allclose(_proj(lib, a, w, bias, 2, base), base + ref, rtol=0, atol=2e-4)


GEMM1 = 0x800   # include/wdr.h WDR_DBG_PROJ_GEMM1


@pytest.mark.parametrize("N", [1280, 2560, 5120])
def test_encoder_gemm_tiles(lib, N):
    """The encoder-batch GEMMs (M >= 4096): k_gemm4 (256 x 256 ping-pong; N = 1280, 2560) and
    k_gemm5 (256 x 128 ping-pong; the wide N = 4d of fc1), a ragged last row tile (M = 4200):
    against the fp64 product
    within the f32 / f16 output rounding, and bit for bit equal to the register-staged k_gemm
    (WDR_DBG_PROJ_GEMM1), whose per-row arithmetic every other GEMM path shares -- every epilogue."""
    rng = np.random.default_rng(N)
    M, K = 4200, 256
    a = rng.standard_normal((M, K)).astype(np.float16).astype(np.float32)
    w = (rng.standard_normal((N, K)) * 0.05).astype(np.float16).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    ref = a.astype(np.float64) @ w.T.astype(np.float64) + bias
    got = _proj(lib, a, w, bias, 3)
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-4)
    np.testing.assert_allclose(_proj(lib, a, w, bias, 1), _gelu(ref), rtol=2e-3, atol=2e-3)
    base = rng.standard_normal((M, N)).astype(np.float32)
    resid = _proj(lib, a, w, bias, 2, base)
    np.testing.assert_allclose(resid, base + ref, rtol=0, atol=2e-4)
    np.testing.assert_array_equal(_proj(lib, a, w, bias, 3 | GEMM1), got)
    np.testing.assert_array_equal(_proj(lib, a, w, bias, 2 | GEMM1, base), resid)
    np.testing.assert_array_equal(_proj(lib, a, w, bias, 0 | GEMM1), _proj(lib, a, w, bias, 0))
    np.testing.assert_array_equal(_proj(lib, a, w, bias, 1 | GEMM1), _proj(lib, a, w, bias, 1))


@pytest.mark.parametrize("M", [300, 1500])
def test_gemm2_tiles_bit_identical(lib, M):
    """k_gemm2 (the 128 x 128 LDS-DMA tile of single-window encodes, M < 4096) with its
    transposed-accumulator vector epilogue: every epilogue bit for bit equal to the reference
    tile k_gemm (WDR_DBG_PROJ_GEMM1), a ragged last row tile included."""
    rng = np.random.default_rng(M + 7)
    K, N = 512, 1280
    a = rng.standard_normal((M, K)).astype(np.float16).astype(np.float32)
    w = (rng.standard_normal((N, K)) * 0.05).astype(np.float16).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    base = rng.standard_normal((M, N)).astype(np.float32)
    for epi in (0, 1, 3):
        np.testing.assert_array_equal(_proj(lib, a, w, bias, epi), _proj(lib, a, w, bias, epi | GEMM1))
    np.testing.assert_array_equal(_proj(lib, a, w, bias, 2, base), _proj(lib, a, w, bias, 2 | GEMM1, base))
    np.testing.assert_array_equal(_proj(lib, a, w, None, 3), _proj(lib, a, w, None, 3 | GEMM1))


ROWS = 0x200   # include/wdr.h WDR_DBG_PROJ_ROWS


@pytest.mark.parametrize("N,K,epi", [(1280, 5120, 2), (1280, 1280, 2), (3840, 1280, 0), (5120, 1280, 1),
                                     (51866, 1280, 3)])
def test_rows_projection_bit_identical_any_m(lib, N, K, epi):
    """The decoder-rows kernel (csrc/rows.h: every decoder projection of steps, prompt prefills
    and DTW re-forwards): a row's result must not depend on how many rows share the launch --
    M = 1 .. 300 rows, one to several row tiles, the narrow (16-column) and wide (32-column)
    tilings, the 16-wave K = 5120 form -- bit for bit, and match the fp64 product."""
    rng = np.random.default_rng(N + K + epi + 1)
    MX = 300
    a = rng.standard_normal((MX, K)).astype(np.float16).astype(np.float32)
    w = (rng.standard_normal((N, K)) * 0.03).astype(np.float16).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    base = rng.standard_normal((MX, N)).astype(np.float32)
    full = _proj(lib, a, w, bias, epi | ROWS, base if epi == 2 else None)
    ref = a[:20].astype(np.float64) @ w.T.astype(np.float64) + bias
    want = {0: ref, 1: _gelu(ref), 2: base[:20] + ref, 3: ref}[epi]
    tol = dict(rtol=0, atol=2e-4) if epi in (2, 3) else dict(rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(full[:20], want, **tol)
    for M in (1, 2, 7, 16, 17, 33, 64, 130):
        got = _proj(lib, a[:M], w, bias, epi | ROWS, base[:M] if epi == 2 else None)
        np.testing.assert_array_equal(got, full[:M], err_msg="M=%d" % M)
    # a row in the middle of a launch equals the same row alone
    one = _proj(lib, a[257:258], w, bias, epi | ROWS, base[257:258] if epi == 2 else None)
    np.testing.assert_array_equal(one, full[257:258])


def test_projection_logits_shape(lib):
    """decoder logits: N not a multiple of the tile (51866 x d), M = 1 (the row kernel)."""
    rng = np.random.default_rng(7)
    K, N = 128, 51866
    a = rng.standard_normal((1, K)).astype(np.float16).astype(np.float32)
    w = (rng.standard_normal((N, K)) * 0.1).astype(np.float16).astype(np.float32)
    ref = a.astype(np.float64) @ w.T.astype(np.float64)
    np.testing.assert_allclose(_proj(lib, a, w, None, 3), ref, rtol=0, atol=2e-4)


def _attn_ref(q, k, v, H, causal):
    Tq, Tk = q.shape[0], k.shape[0]
    out = np.zeros((Tq, H * 64))
    for h in range(H):
        s = q[:, h * 64:(h + 1) * 64].astype(np.float64) @ k[:, h * 64:(h + 1) * 64].T.astype(np.float64) / 8.0
        if causal:
            s = s + np.triu(np.full((Tq, Tk), -np.inf), 1)
        p = np.exp(s - s.max(1, keepdims=True))
        p /= p.sum(1, keepdims=True)
        out[:, h * 64:(h + 1) * 64] = p @ v[:, h * 64:(h + 1) * 64]
    return out


@pytest.mark.parametrize("Tq,Tk,H,causal", [(1500, 1500, 2, 0), (37, 1500, 3, 0), (129, 129, 2, 1), (5, 5, 1, 1)])
def test_flash_attention_matches_fp32_reference(lib, Tq, Tk, H, causal):
    rng = np.random.default_rng(Tq + Tk)
    q = (rng.standard_normal((Tq, H * 64)) * 1.0).astype(np.float16)
    k = (rng.standard_normal((Tk, H * 64)) * 1.0).astype(np.float16)
    v = rng.standard_normal((Tk, H * 64)).astype(np.float16)
    out = np.zeros((Tq, H * 64), np.float32)
    _lib.check(lib.wdr_dbg_attn(q.view(np.uint16).ctypes.data_as(U16), k.view(np.uint16).ctypes.data_as(U16),
                                v.view(np.uint16).ctypes.data_as(U16), Tq, Tk, H, causal, out.ctypes.data_as(F32)))
    ref = _attn_ref(q.astype(np.float32), k.astype(np.float32), v.astype(np.float32), H, causal)
    # P enters P.V as f16 (as in ggml), output rounded to f16
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-2)
    assert np.abs(out - ref).mean() < 1.5e-3


def _xattn(lib, q, kv, H, row_slot=None, grp=None, iters=1):
    R = q.shape[0]
    out = np.zeros((R, H * 64), np.float32)
    rs = None if row_slot is None else np.ascontiguousarray(row_slot, np.int32)
    g = None if grp is None else np.ascontiguousarray(grp, np.int32)
    _lib.check(lib.wdr_dbg_xattn(_f16bits(q).ctypes.data_as(U16), _f16bits(kv).ctypes.data_as(U16),
                                 None if rs is None else rs.ctypes.data_as(I32),
                                 None if g is None else g.ctypes.data_as(I32), R, kv.shape[0], H, iters,
                                 out.ctypes.data_as(F32)))
    return out


@pytest.mark.parametrize("H", [3, 4])
def test_decode_cross_attention(lib, H):
    """k_xattn_partial + k_xattn_combine (64-key chunks, row groups sharing a chunk): per-row
    slots (batched greedy step: two heads per workgroup when the head count is even), beam
    groups sharing a slot, the shared form, and repeated launches.  Every row must equal the
    fp64 attention within the f16 P / output rounding, and a row's result must not depend on
    the group -- or the kernel -- it is computed in (batch composition varies with timing)."""
    rng = np.random.default_rng(11)
    S, R = 6, 24
    q = (rng.standard_normal((R, H * 64)) * 1.5).astype(np.float16).astype(np.float32)
    kv = rng.standard_normal((S, 1500, 2 * H * 64)).astype(np.float16).astype(np.float32)
    slot = rng.integers(0, S, R)
    ref = np.concatenate([_attn_ref(q[r:r + 1], kv[slot[r], :, :H * 64], kv[slot[r], :, H * 64:], H, 0)
                          for r in range(R)])
    rows = _xattn(lib, q, kv, H, slot)
    np.testing.assert_allclose(rows, ref, rtol=0, atol=1e-2)
    assert np.abs(rows - ref).mean() < 1.5e-3
    # groups: rows of a group share the leader's slot
    sizes = [5, 1, 3, 8, 2, 5]
    grp, gslot = np.zeros(R, np.int32), np.zeros(R, np.int64)
    r0 = 0
    for i, n in enumerate(sizes):
        grp[r0] = n
        gslot[r0:r0 + n] = i % S
        r0 += n
    assert r0 == R
    gref = np.concatenate([_attn_ref(q[r:r + 1], kv[gslot[r], :, :H * 64], kv[gslot[r], :, H * 64:], H, 0)
                           for r in range(R)])
    grouped = _xattn(lib, q, kv, H, gslot, grp)
    np.testing.assert_allclose(grouped, gref, rtol=0, atol=1e-2)
    single = _xattn(lib, q, kv, H, gslot)   # same rows, every row its own group
    np.testing.assert_array_equal(grouped, single)
    np.testing.assert_array_equal(_xattn(lib, q, kv, H, gslot, grp, iters=3), grouped)
    # shared K/V (one segment's beams on a State's own step), R <= 8
    shared = _xattn(lib, q[:5], kv[:1], H)
    np.testing.assert_array_equal(shared, _xattn(lib, q[:5], kv[:1], H, np.zeros(5), [5, 0, 0, 0, 0]))
    np.testing.assert_allclose(shared, _attn_ref(q[:5], kv[0, :, :H * 64], kv[0, :, H * 64:], H, 0), rtol=0,
                               atol=1e-2)


def test_decode_cross_attention_mma_tiles(lib):
    """The decoder-rows cross-attention of prompt prefills / DTW re-forwards (groups above 8
    rows): MFMA row tiles of <= 128 rows (k_xattn_mma) beside VALU groups, merged by one
    combine.  Every row matches the fp64 attention; a row's result does not depend on its
    group's size or tile (a 40-row group equals the same rows as a 12 + 28 split, and a 200-row
    group spans two tiles)."""
    rng = np.random.default_rng(17)
    H, S = 4, 3
    sizes = [40, 3, 200, 1, 12]
    R = sum(sizes)
    q = (rng.standard_normal((R, H * 64)) * 1.5).astype(np.float16).astype(np.float32)
    kv = rng.standard_normal((S, 1500, 2 * H * 64)).astype(np.float16).astype(np.float32)
    grp, slot = np.zeros(R, np.int32), np.zeros(R, np.int64)
    r0 = 0
    for i, n in enumerate(sizes):
        grp[r0] = n
        slot[r0:r0 + n] = i % S
        r0 += n
    got = _xattn(lib, q, kv, H, slot, grp)
    pick = list(range(0, 40, 7)) + [40, 42] + list(range(43, 243, 37)) + [243, 244, 255]
    ref = np.concatenate([_attn_ref(q[r:r + 1], kv[slot[r], :, :H * 64], kv[slot[r], :, H * 64:], H, 0)
                          for r in pick])
    np.testing.assert_allclose(got[pick], ref, rtol=0, atol=1e-2)
    assert np.abs(got[pick] - ref).mean() < 1.5e-3
    split = grp.copy()
    split[0], split[12] = 12, 28
    np.testing.assert_array_equal(_xattn(lib, q, kv, H, slot, split), got)


def test_signal_energy_is_bit_exact(lib):
    rng = np.random.default_rng(0)
    for n in (1, 64, 65, 1000, 160000):
        x = (rng.standard_normal(n) * 0.2).astype(np.float32)
        out = np.zeros(n, np.float32)
        _lib.check(lib.wdr_dbg_energy(x.ctypes.data_as(F32), n, out.ctypes.data_as(F32)))
        np.testing.assert_array_equal(out, omel.signal_energy(x))


def _dtw_dp(lib, x, seek):
    x = np.ascontiguousarray(x, np.float32)
    rows, cols = x.shape
    t = np.zeros(rows + 8, np.int32)
    nt = C.c_int32()
    _lib.check(lib.wdr_dbg_dtw_dp(x.ctypes.data_as(F32), rows, cols, seek, t.ctypes.data_as(I32), C.byref(nt)))
    return list(t[:nt.value])


def test_dtw_dp_bit_exact_against_golden_including_ties(lib):
    import os
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "dtw_cases.npz"))
    for key in [k for k in g.files if k.startswith("x")]:
        x = g[key]
        ti, tj = g["ti" + key[1:]], g["tj" + key[1:]]
        want, last = [], 0
        for v, t in zip(ti.tolist(), tj.tolist()):
            if v != last:
                want.append(2 * t + 100)
                last = v
        assert _dtw_dp(lib, x, 100) == want, key


def test_dtw_dp_max_size(lib):
    rng = np.random.default_rng(5)
    x = rng.standard_normal((221, 1500)).astype(np.float32)
    assert _dtw_dp(lib, x, 0) == odtw.token_times(x, 0)
    x = np.round(rng.standard_normal((40, 1500))).astype(np.float32)   # ties everywhere
    assert _dtw_dp(lib, x, 3000) == odtw.token_times(x, 3000)


def test_dtw_preprocessing_bit_exact(lib):
    rng = np.random.default_rng(9)
    A, N, n_audio, sot_len = 5, 23, 731, 1
    logits = rng.standard_normal((A, N, 1500)).astype(np.float32) * 3
    cap = np.exp(logits - logits.max(-1, keepdims=True))
    cap = (cap / cap.sum(-1, keepdims=True)).astype(np.float32)
    rows = N - sot_len - 1
    x = np.zeros((rows, n_audio), np.float32)
    t = np.zeros(N + 8, np.int32)
    nt = C.c_int32()
    _lib.check(lib.wdr_dbg_dtw(cap.ctypes.data_as(F32), A, N, n_audio, sot_len, 200, x.ctypes.data_as(F32),
                               t.ctypes.data_as(I32), C.byref(nt)))
    xr = odtw.alignment_matrix(cap, 2 * n_audio, sot_len)
    np.testing.assert_array_equal(x, xr)
    assert list(t[:nt.value]) == odtw.token_times(xr, 200)


def _e4m3_decode(b):
    """OCP e4m3fn byte -> float (sign, 4-bit exponent bias 7, 3-bit mantissa, no infinities)."""
    b = np.asarray(b, np.uint8).astype(np.int32)
    s = np.where(b & 0x80, -1.0, 1.0)
    e = (b >> 3) & 0xF
    m = (b & 7).astype(np.float64)
    v = np.where(e == 0, m / 8.0 * 2.0 ** -6, (1 + m / 8.0) * 2.0 ** (e - 7))
    v = np.where((e == 15) & ((b & 7) == 7), np.nan, v)
    return s * v


def _e4m3_grid():
    g = _e4m3_decode(np.arange(256))
    return np.unique(g[np.isfinite(g)])


@pytest.mark.parametrize("M,N,K,epi", [(300, 256, 256, 3), (1500, 1280, 1280, 2), (777, 3840, 1280, 0),
                                       (600, 1280, 5120, 2), (256, 5120, 1280, 1)])
def test_fp8_projection(lib, M, N, K, epi):
    """fp8 encoder GEMM (BASELINE configs[4]): the per-row e4m3 quantisation is round-to-nearest
    onto the e4m3 grid at scale max|row| / 448, and the GEMM output equals the fp64 product of
    the dequantised operands (scales applied in the epilogue) within f32 accumulation error,
    for both tile widths (N = 1280: 128-column tiles) and every epilogue."""
    rng = np.random.default_rng(M + N + K)
    a = (rng.standard_normal((M, K)) * rng.uniform(0.1, 3.0, (M, 1))).astype(np.float16)
    w = (rng.standard_normal((N, K)) * 0.05).astype(np.float16)
    bias = (rng.standard_normal(N) * 0.1).astype(np.float32)
    base = rng.standard_normal((M, N)).astype(np.float32)
    out = base.copy() if epi == 2 else np.zeros((M, N), np.float32)
    a8, w8 = np.zeros((M, K), np.uint8), np.zeros((N, K), np.uint8)
    asc, wsc = np.zeros(M, np.float32), np.zeros(N, np.float32)
    U8 = C.POINTER(C.c_uint8)
    _lib.check(lib.wdr_dbg_proj_fp8(a.view(np.uint16).ctypes.data_as(U16), w.view(np.uint16).ctypes.data_as(U16),
                                    bias.ctypes.data_as(F32), M, N, K, epi, out.ctypes.data_as(F32),
                                    a8.ctypes.data_as(U8), asc.ctypes.data_as(F32), w8.ctypes.data_as(U8),
                                    wsc.ctypes.data_as(F32)))
    # quantisation: scale and nearest grid point (ties may go either way: within half a step)
    np.testing.assert_allclose(asc, np.abs(a.astype(np.float32)).max(1) / 448, rtol=1e-6)
    grid = _e4m3_grid()
    x = a.astype(np.float64) / asc[:, None].astype(np.float64)
    q = _e4m3_decode(a8)
    idx = np.clip(np.searchsorted(grid, x), 1, len(grid) - 1)
    nearest = np.minimum(np.abs(grid[idx] - x), np.abs(grid[idx - 1] - x))
    # x is computed here in f64 (the kernel multiplies by 448 / amax in f32): near-ties may round
    # to the other neighbour
    excess = np.abs(q - x) - nearest
    bad = excess > 1e-5 * np.maximum(np.abs(x), 1.0)
    assert not bad.any(), (int(bad.sum()), float(excess.max()), x[bad][:5], q[bad][:5])
    # GEMM on the dequantised operands
    A = _e4m3_decode(a8) * asc[:, None]
    W = _e4m3_decode(w8) * wsc[:, None]
    ref = A @ W.T + bias
    want = {0: ref, 1: _gelu(ref), 2: base + ref, 3: ref}[epi]
    tol = dict(rtol=2e-3, atol=2e-3) if epi in (0, 1) else dict(rtol=0, atol=1e-4 * np.abs(A).max() * np.abs(W).max() * K ** 0.5 + 1e-4)
    np.testing.assert_allclose(out, want, **tol)
    # and close to the f16 product (the quantisation error, e4m3 has 3 mantissa bits)
    f16ref = a.astype(np.float64) @ w.T.astype(np.float64) + bias
    rel = np.linalg.norm(ref - f16ref) / np.linalg.norm(f16ref)
    assert rel < 0.06, rel
