"""Cross-attention DTW token alignment (oracle side).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates whisper.cpp `whisper_exp_compute_token_level_timestamps_dtw`,
`median_filter` and `dtw_and_backtrace` (enabled by `enable_dtw`,
src/engine.rs:24, preset chosen at src/transcribe.rs:117-129; SURVEY.md §8(a)
a12, Appendix A.6):

  w[h][tok][frame] = softmax(QK^T) of the alignment heads (all 1500 columns),
  truncated to n_frames/2 columns (no re-softmax);
  normalise over tokens per (head, column): (x - mean) / sqrt(var + 1e-9);
  median filter width 7 along columns with reflect padding;
  mean over heads, negate; keep token rows [sot_len, N-1);
  DTW (j outer, i inner; strict-< ties: diag, up, else left); backtrace;
  t_dtw = 2 * frame + seek for each change of the token index along the path.

The DTW recurrence / backtrace and the median filter are pinned against
transformers' `_dynamic_time_warping` / `_median_filter` (tests/golden).
"""
from __future__ import annotations

import numpy as np


def norm_over_tokens(w: np.ndarray, eps: float = 1e-9) -> np.ndarray:
    """w: [H][N][M]; ggml_norm (f32) along the token axis for every (head, column):
    mean = float(double sum / N); v = x - mean; var = float(double sum of f32 v*v / N);
    scale = 1 / sqrtf(var + eps); y = v * scale.  Sums run in token order."""
    w = w.astype(np.float32)
    H, N, M = w.shape
    s = np.zeros((H, M), np.float64)
    for t in range(N):
        s += w[:, t, :].astype(np.float64)
    mean = (s / N).astype(np.float32)
    s2 = np.zeros((H, M), np.float64)
    for t in range(N):
        v = (w[:, t, :] - mean).astype(np.float32)
        s2 += (v * v).astype(np.float32).astype(np.float64)
    var = (s2 / N).astype(np.float32)
    scale = (np.float32(1.0) / np.sqrt((var + np.float32(eps)).astype(np.float32))).astype(np.float32)
    return ((w - mean[:, None, :]).astype(np.float32) * scale[:, None, :]).astype(np.float32)


def median_filter(w: np.ndarray, width: int = 7) -> np.ndarray:
    """Median along the last axis, reflect padding idx<0 -> -idx, idx>=M -> 2(M-1)-idx."""
    M = w.shape[-1]
    half = width // 2
    idx = np.arange(M)[:, None] + np.arange(-half, half + 1)[None, :]
    idx = np.where(idx < 0, -idx, idx)
    idx = np.where(idx >= M, 2 * (M - 1) - idx, idx)
    win = w[..., idx]                       # [..., M, width]
    return np.sort(win, axis=-1)[..., half]


def dtw_cost_matrix(x: np.ndarray):
    """x: [N][M] f32.  Returns (cost[N+1][M+1] f32, trace[N+1][M+1] int8)."""
    N, M = x.shape
    cost = np.full((N + 1, M + 1), np.inf, np.float32)
    trace = np.full((N + 1, M + 1), -1, np.int8)
    cost[0, 0] = 0.0
    for j in range(1, M + 1):
        for i in range(1, N + 1):
            c0, c1, c2 = cost[i - 1, j - 1], cost[i - 1, j], cost[i, j - 1]
            if c0 < c1 and c0 < c2:
                c, t = c0, 0
            elif c1 < c0 and c1 < c2:
                c, t = c1, 1
            else:
                c, t = c2, 2
            cost[i, j] = np.float32(x[i - 1, j - 1] + c)
            trace[i, j] = t
    return cost, trace


def dtw_cost_matrix_fast(x: np.ndarray):
    """Same recurrence, vectorised along anti-diagonals (identical results: each cell
    depends only on the previous two anti-diagonals)."""
    N, M = x.shape
    cost = np.full((N + 1, M + 1), np.inf, np.float32)
    trace = np.full((N + 1, M + 1), -1, np.int8)
    cost[0, 0] = 0.0
    x = x.astype(np.float32)
    for s in range(2, N + M + 1):
        i = np.arange(max(1, s - M), min(N, s - 1) + 1)
        j = s - i
        c0, c1, c2 = cost[i - 1, j - 1], cost[i - 1, j], cost[i, j - 1]
        t = np.where((c0 < c1) & (c0 < c2), 0, np.where((c1 < c0) & (c1 < c2), 1, 2)).astype(np.int8)
        c = np.where(t == 0, c0, np.where(t == 1, c1, c2))
        cost[i, j] = (x[i - 1, j - 1] + c).astype(np.float32)
        trace[i, j] = t
    return cost, trace


def backtrace(trace: np.ndarray):
    trace = trace.copy()
    N1, M1 = trace.shape
    trace[0, :] = 2
    trace[:, 0] = 1
    i, j = N1 - 1, M1 - 1
    ti, tj = [], []
    while i > 0 or j > 0:
        ti.append(i - 1)
        tj.append(j - 1)
        t = trace[i, j]
        if t == 0:
            i -= 1
            j -= 1
        elif t == 1:
            i -= 1
        elif t == 2:
            j -= 1
        else:
            raise RuntimeError("bad trace")
    return np.array(ti[::-1], np.int32), np.array(tj[::-1], np.int32)


def dtw(x: np.ndarray):
    _, trace = dtw_cost_matrix_fast(x)
    return backtrace(trace)


def alignment_matrix(qk: np.ndarray, n_frames: int, sot_len: int, medfilt: int = 7) -> np.ndarray:
    """qk: [H][N_tok][1500] post-softmax alignment-head attention.  Returns the
    [N_tok - sot_len - 1][n_frames//2] matrix DTW runs on (ggml_mean: double sum over
    heads in head order, cast to float, / H, then scaled by -1)."""
    n_audio = n_frames // 2
    w = qk[:, :, :n_audio]
    w = norm_over_tokens(w)
    w = median_filter(w, medfilt)
    s = np.zeros(w.shape[1:], np.float64)
    for h in range(w.shape[0]):
        s += w[h].astype(np.float64)
    w = ((s.astype(np.float32) / np.float32(w.shape[0])) * np.float32(-1.0)).astype(np.float32)
    return w[sot_len:w.shape[0] - 1]


def token_times(x: np.ndarray, seek: int):
    """DTW over x; returns the list of t_dtw (centiseconds) for text tokens, in order:
    one entry per change of the token index along the path (starting from last_v = 0)."""
    ti, tj = dtw(x)
    out = []
    last_v = 0
    for v, t in zip(ti.tolist(), tj.tolist()):
        if v != last_v:
            out.append(2 * t + seek)
            last_v = v
    return out
