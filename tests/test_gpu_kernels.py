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


def _proj_ln(lib, x, g, b, w, bias, epi, fused):
    M, K = x.shape
    N = w.shape[0]
    out = np.zeros((M, N), np.float32)
    xc, gc, bc = (np.ascontiguousarray(v, np.float32) for v in (x, g, b))
    wb = _f16bits(w)
    bb = np.ascontiguousarray(bias, np.float32)
    _lib.check(lib.wdr_dbg_proj_ln(xc.ctypes.data_as(F32), gc.ctypes.data_as(F32), bc.ctypes.data_as(F32),
                                   wb.ctypes.data_as(U16), bb.ctypes.data_as(F32), M, N, K, epi, int(fused),
                                   out.ctypes.data_as(F32)))
    return out


@pytest.mark.parametrize("N,epi", [(3840, 0), (1280, 0), (5120, 1), (51866, 3)])
def test_rows_ln_fused_equals_split(lib, N, epi):
    """rows_forward normalises the projection's input rows inside the row kernel up to 64 rows
    (csrc/rows.cpp; every batched step and prompt prefill of the step batcher): LayerNorm fused
    into the prologue -- 16-row tiles on the narrow projections (qkv 3d, xq d), 32-row tiles on
    fc1 (4d, GELU) and the logits (V) -- must equal the separate k_layernorm launch into f16 rows
    followed by the same projection, bit for bit, at R = 1 .. 64 (16, 48 and 64 among them)."""
    rng = np.random.default_rng(N + epi)
    K = 1280
    x = (rng.standard_normal((64, K)) * 2.0 + 0.3).astype(np.float32)
    g = (1.0 + 0.1 * rng.standard_normal(K)).astype(np.float32)
    b = (0.1 * rng.standard_normal(K)).astype(np.float32)
    w = (rng.standard_normal((N, K)) * 0.03).astype(np.float16).astype(np.float32)
    bias = (rng.standard_normal(N) * 0.1).astype(np.float32)
    for M in (1, 16, 17, 33, 48, 64):
        fused = _proj_ln(lib, x[:M], g, b, w, bias, epi, True)
        split = _proj_ln(lib, x[:M], g, b, w, bias, epi, False)
        np.testing.assert_array_equal(fused, split, err_msg="M=%d" % M)
    # and against an fp64 LayerNorm + projection
    xm = x[:16].astype(np.float64)
    ln = (xm - xm.mean(1, keepdims=True)) / np.sqrt(xm.var(1, keepdims=True) + 1e-5) * g + b
    ref = ln.astype(np.float16).astype(np.float64) @ w.T.astype(np.float64) + bias
    want = _gelu(ref) if epi == 1 else ref
    np.testing.assert_allclose(fused[:16], want, rtol=2e-3, atol=3e-3)


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


def test_dtw_dp_wave_form_boundaries(lib):
    # the one-wave DP (<= 64 token rows, kernels/elem.hip k_dtw_dp_wave) and the 256-thread form
    # (above 64) at their edges: one row / one column, exactly 64 and 65 rows, short and full
    # windows, tie-heavy integer costs -- token times identical to the oracle's DP
    rng = np.random.default_rng(11)
    for rows, cols, ties in [(1, 1, False), (1, 1500, False), (3, 2, True), (64, 7, True), (64, 1500, False),
                             (65, 300, True), (63, 1500, True), (17, 333, False)]:
        x = rng.standard_normal((rows, cols)).astype(np.float32)
        if ties:
            x = np.round(x)
        assert _dtw_dp(lib, x, 40) == odtw.token_times(x, 40), (rows, cols, ties)


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


def _mx_exp(amax):
    """E8M0 exponent of an F8 block (k_gemm8's f8_block_exp): the smallest e with amax / 2^e <=
    448, amax = m 2^x (m in [0.5, 1)): x - 9 if m <= 0.875 else x - 8, clamped to [-126, 126]."""
    m, x = np.frexp(amax.astype(np.float32))
    e = np.where(m <= 0.875, x - 9, x - 8)
    return np.where(amax > 0, np.clip(e, -126, 126), -126)


def _mx_check(x, q8, sc):
    """x [R][K] f64 values, q8 [R][K] e4m3 bytes, sc [R][K/32] E8M0 bytes: each block's scale is
    _mx_exp of its max |x|, and each byte the nearest e4m3 value of x / 2^e (ties either way)."""
    R, K = x.shape
    xb = x.reshape(R, K // 32, 32)
    e = _mx_exp(np.abs(xb).max(-1))
    np.testing.assert_array_equal(sc.astype(np.int64) - 127, e)
    y = (xb / np.exp2(e)[..., None]).reshape(R, K)
    assert np.abs(y).max() <= 448
    grid = _e4m3_grid()
    q = _e4m3_decode(q8)
    idx = np.clip(np.searchsorted(grid, y), 1, len(grid) - 1)
    nearest = np.minimum(np.abs(grid[idx] - y), np.abs(grid[idx - 1] - y))
    excess = np.abs(q - y) - nearest
    bad = excess > 1e-5 * np.maximum(np.abs(y), 1.0)
    assert not bad.any(), (int(bad.sum()), float(excess.max()), y[bad][:5], q[bad][:5])


def _mx_dequant(q8, sc):
    R, K = q8.shape
    return (_e4m3_decode(q8).reshape(R, K // 32, 32) * np.exp2(sc.astype(np.float64) - 127)[..., None]).reshape(R, K)


@pytest.mark.parametrize("M,N,K,epi", [(300, 256, 256, 3), (1500, 1280, 1280, 2), (777, 3840, 1280, 0),
                                       (600, 1280, 5120, 2), (256, 5120, 1280, 1), (333, 512, 1280, 7)])
def test_fp8_projection(lib, M, N, K, epi):
    """fp8 encoder GEMM (BASELINE configs[4], k_gemm8, MX): every row of both operands is e4m3
    with one E8M0 scale per 32 k -- the smallest power of two that maps the block's max |x| to
    <= 448, the values rounded to nearest -- and the GEMM output equals the fp64 product of the
    dequantised operands (the scales applied inside the block-scaled MFMA) within f32
    accumulation error, for every epilogue, row counts off the 256-row tile (rows past M read as
    zeros through the buffer descriptor) and the GELU -> e4m3 epilogue that feeds fc2 (7: its
    output blocks are checked like the inputs)."""
    rng = np.random.default_rng(M + N + K)
    a = (rng.standard_normal((M, K)) * rng.uniform(0.1, 3.0, (M, 1))).astype(np.float16)
    a[:, :32] *= np.float16(0.01)   # blocks of very different magnitude in one row
    w = (rng.standard_normal((N, K)) * 0.05).astype(np.float16)
    bias = (rng.standard_normal(N) * 0.1).astype(np.float32)
    base = rng.standard_normal((M, N)).astype(np.float32)
    out = base.copy() if epi == 2 else np.zeros((M, N), np.float32)
    a8, w8 = np.zeros((M, K), np.uint8), np.zeros((N, K), np.uint8)
    asc, wsc = np.zeros((M, K // 32), np.uint8), np.zeros((N, K // 32), np.uint8)
    U8 = C.POINTER(C.c_uint8)
    _lib.check(lib.wdr_dbg_proj_fp8(a.view(np.uint16).ctypes.data_as(U16), w.view(np.uint16).ctypes.data_as(U16),
                                    bias.ctypes.data_as(F32), M, N, K, epi, out.ctypes.data_as(F32),
                                    a8.ctypes.data_as(U8), asc.ctypes.data_as(U8), w8.ctypes.data_as(U8),
                                    wsc.ctypes.data_as(U8)))
    _mx_check(a.astype(np.float64), a8, asc)
    _mx_check(w.astype(np.float64), w8, wsc)
    A, W = _mx_dequant(a8, asc), _mx_dequant(w8, wsc)
    ref = A @ W.T + bias
    if epi == 7:
        g = _gelu(ref)
        gb = g.reshape(M, N // 32, 32)
        # the kernel rounded its f32 GELU to e4m3 at its block's scale: half an ulp, 2^-4
        # relative in the normal range, 2^(e-10) absolute in the subnormal one (x2: the kernel's
        # block max may round to the neighbouring exponent)
        e = _mx_exp(np.abs(gb).max(-1))[..., None]
        err = np.abs(out.reshape(M, N // 32, 32) - gb)
        bound = 2 * np.maximum(np.abs(gb) * 2.0 ** -4, np.exp2(e - 10.0)) + 1e-5 * np.abs(gb).max()
        assert (err <= bound).all(), float((err / bound).max())
        return
    want = {0: ref, 1: _gelu(ref), 2: base + ref, 3: ref}[epi]
    tol = dict(rtol=2e-3, atol=2e-3) if epi in (0, 1) else dict(rtol=0, atol=1e-4 * np.abs(A).max() * np.abs(W).max() * K ** 0.5 + 1e-4)
    np.testing.assert_allclose(out, want, **tol)
    # and close to the f16 product (the quantisation error, e4m3 has 3 mantissa bits)
    f16ref = a.astype(np.float64) @ w.T.astype(np.float64) + bias
    rel = np.linalg.norm(ref - f16ref) / np.linalg.norm(f16ref)
    assert rel < 0.06, rel


def test_mfma_scale_lane_map(lib):
    """The lane maps k_gemm8 relies on for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3), measured:
    lane l (g = l >> 4) holds k = 16g .. 16g+15 of row (A) / column (B) l & 15 in its bytes 0-15
    and k = 64+16g .. +15 in bytes 16-31, and its scale register (op_sel 0: byte 0) scales the
    k-block g (k = 32g .. 32g+31) of that row / column: out[m][n] = sum_k 2^(sa[16 (k/32)+m]-127)
    2^(sb[16 (k/32)+n]-127) A[m][k] B[k][n].  (A first hypothesis, bytes 0-31 = k 32g .. 32g+31,
    failed the "data" case: 80 where it predicts 64.)  Exact small integers, asymmetric patterns."""
    U8 = C.POINTER(C.c_uint8)
    I32 = C.POINTER(C.c_int32)
    one = 0x38                                   # e4m3 1.0
    rng = np.random.default_rng(7)
    vals = np.array([0x30, 0x38, 0x40, 0x44, 0xb8, 0x00], np.uint8)   # 0.5, 1, 2, 3, -1, 0
    cases = []
    for name in ("blocks", "rows", "data", "random"):
        a = np.full((64, 32), one, np.uint8)
        b = np.full((64, 32), one, np.uint8)
        sa = np.full(64, 127, np.int32)
        sb = np.full(64, 127, np.int32)
        if name == "blocks":
            sa = 127 + (np.arange(64) >> 4)
        elif name == "rows":
            sa = 127 + (np.arange(64) & 3)
            sb = 127 - (np.arange(64) & 1)
        elif name == "data":
            a[(np.arange(64) >> 4) != 1] = 0
            sa = 127 + (np.arange(64) >> 4)
        else:
            a = vals[rng.integers(0, len(vals), (64, 32))]
            b = vals[rng.integers(0, len(vals), (64, 32))]
            sa = (127 + rng.integers(-3, 4, 64)).astype(np.int32)
            sb = (127 + rng.integers(-3, 4, 64)).astype(np.int32)
        out = np.zeros((64, 4), np.float32)
        _lib.check(lib.wdr_dbg_mfma_scale(a.ctypes.data_as(U8), b.ctypes.data_as(U8), sa.astype(np.int32).ctypes.data_as(I32),
                                          sb.astype(np.int32).ctypes.data_as(I32), out.ctypes.data_as(F32)))
        A = _e4m3_decode(a)                      # [lane][byte]
        Bv = _e4m3_decode(b)
        want = np.zeros((16, 16))
        for m in range(16):
            for n in range(16):
                for g in range(4):
                    for j in range(32):
                        k = 16 * g + j if j < 16 else 64 + 16 * g + (j - 16)
                        blk = k // 32
                        want[m, n] += (2.0 ** (sa[16 * blk + m] - 127) * 2.0 ** (sb[16 * blk + n] - 127) *
                                       float(A[16 * g + m, j] * Bv[16 * g + n, j]))
        got = np.zeros((16, 16))
        for l in range(64):
            for r in range(4):
                got[(l >> 4) * 4 + r, l & 15] = out[l, r]
        cases.append((name, got, want))
    for name, got, want in cases:
        assert np.array_equal(got, want), (name, got[:4, :4], want[:4, :4])
