"""DTW near-tie analysis shared by tests/test_gpu_baseline_models.py and tools/dtw_diag.py.

For one DTW re-forward (whisper.cpp whisper_exp_compute_token_level_timestamps_dtw, run for the
window by state.full, src/transcribe.rs:389) given the oracle's and the GPU's alignment-head
probabilities for the SAME window and token sequence:
  * path margin = cost_o(path_g) - cost_o(path_o): how much worse the GPU's DTW path is under the
    ORACLE's alignment matrix (0 when the paths agree);
  * perturbation = sum over both paths' cells of |x_g - x_o|: the matrix difference the capture
    error put on those paths.
An anchor that moved with margin <= perturbation sits at a near-tie: both paths are optimal within
the capture's f16-rounding-level error, and neither side is wrong.
"""
from __future__ import annotations

import numpy as np

from oracle import dtw as odtw
from oracle.model import DecoderState
from oracle.vocab import LANGS


def _anchors(ti, tj, seek):
    out, last = [], 0
    for v, t in zip(ti.tolist(), tj.tolist()):
        if v != last:
            out.append(2 * t + seek)
            last = v
    return out


def analyse(qk_o, qk_g, n_frames, sot_len, seek):
    x_o = odtw.alignment_matrix(qk_o, n_frames, sot_len)
    x_g = odtw.alignment_matrix(qk_g, n_frames, sot_len)
    ti_o, tj_o = odtw.dtw(x_o)
    ti_g, tj_g = odtw.dtw(x_g)
    ko = (ti_o >= 0) & (tj_o >= 0)
    kg = (ti_g >= 0) & (tj_g >= 0)
    cost_oo = float(x_o[ti_o[ko], tj_o[ko]].astype(np.float64).sum())
    cost_og = float(x_o[ti_g[kg], tj_g[kg]].astype(np.float64).sum())
    d = np.abs(x_g - x_o)
    pert = float(d[ti_o[ko], tj_o[ko]].sum() + d[ti_g[kg], tj_g[kg]].sum())
    a_o, a_g = _anchors(ti_o, tj_o, seek), _anchors(ti_g, tj_g, seek)
    moved = [(k, ao, ag) for k, (ao, ag) in enumerate(zip(a_o, a_g)) if ao != ag]
    return dict(anchors_oracle=a_o, anchors_gpu=a_g, moved=moved, path_cost=cost_oo, path_margin=cost_og - cost_oo,
                perturbation=pert, x_spread=float(x_o.std()), cap_rel_max=float(np.abs(qk_g - qk_o).max() /
                                                                              np.abs(qk_o).max()))


def record_dtw_calls(st, model):
    """Wraps WhisperState.dtw_timestamps so that every DTW re-forward of the oracle's state.full
    records (seek, n_frames, sot_len, tokens, qk_o)."""
    calls = []
    orig = st.dtw_timestamps

    def rec(i_segment, n_segments, seek, n_frames, cross, language):
        v = st.v
        toks = [v.sot] + ([v.token_lang(LANGS.index(language))] if v.multilingual else [])
        sot_len = len(toks)
        toks.append(v.not_)
        for s in st.result_all[i_segment:i_segment + n_segments]:
            toks += [t.id for t in s.tokens if t.id < v.eot]
        toks.append(v.eot)
        orig(i_segment, n_segments, seek, n_frames, cross, language)
        _, qk = DecoderState(model).forward(toks, cross, want_logits=None, aheads=st.aheads)
        calls.append(dict(seek=seek, n_frames=n_frames, sot_len=sot_len, tokens=toks, qk_o=qk))

    st.dtw_timestamps = rec
    return calls


def gpu_capture(ctx, x, call, n_aheads):
    """The GPU's alignment-head probabilities for a recorded call: the window's GPU log-mel and
    encoder, then the capture re-forward over the same tokens (wdr_dbg_capture)."""
    ctx.encode(ctx.log_mel_window(x, call["seek"]))
    return ctx.capture(call["tokens"], n_aheads)


def anchored_path(x, entries):
    """The cheapest DTW path through x ([rows][cols], cost = sum of the cells it visits) that
    enters row r at frame entries[r - 1] (row 0 at frame 0): the GPU's DTW times pin where each
    token row starts; within a row the path moves right, between rows down (same frame) or
    diagonally (next frame), so each row's last frame is its successor's entry or the frame
    before it, whichever is cheaper.  Returns (ti, tj) or None if the entries are not monotone."""
    rows, cols = x.shape
    e = [0] + [int(v) for v in entries]
    if len(e) != rows or any(b < a for a, b in zip(e, e[1:])) or e[-1] >= cols:
        return None
    ti, tj = [], []
    for r in range(rows):
        if r + 1 < rows:
            nxt = e[r + 1]
            f = nxt if (nxt == e[r] or x[r, nxt] < 0 or nxt - 1 < e[r]) else nxt - 1
        else:
            f = cols - 1
        for j in range(e[r], f + 1):
            ti.append(r)
            tj.append(j)
    return np.array(ti, np.int32), np.array(tj, np.int32)


def analyse_anchors(qk_o, qk_g, n_frames, sot_len, seek, t_gpu):
    """analyse() for a DTW result known only by its token times (the pipeline's t_dtw of the
    window's text tokens, t = 2 * entry frame + seek): the GPU's path is the cheapest path
    through those entries under the ORACLE's matrix; path margin = its cost - the oracle path's
    cost, perturbation = sum over both paths' cells of |x_g - x_o| (x_g from the GPU's capture
    qk_g).  margin <= perturbation: the GPU's times are optimal within the capture error."""
    x_o = odtw.alignment_matrix(qk_o, n_frames, sot_len)
    x_g = odtw.alignment_matrix(qk_g, n_frames, sot_len)
    ti_o, tj_o = odtw.dtw(x_o)
    a_o = _anchors(ti_o, tj_o, seek)
    p = anchored_path(x_o, [(t - seek) // 2 for t in t_gpu])
    if p is None:
        return dict(anchors_oracle=a_o, anchors_gpu=list(t_gpu), moved=None, path_margin=np.inf, perturbation=0.0)
    ti_g, tj_g = p
    cost_oo = float(x_o[ti_o, tj_o].astype(np.float64).sum())
    cost_og = float(x_o[ti_g, tj_g].astype(np.float64).sum())
    d = np.abs(x_g - x_o)
    pert = float(d[ti_o, tj_o].sum() + d[ti_g, tj_g].sum())
    moved = [(k, ao, ag) for k, (ao, ag) in enumerate(zip(a_o, t_gpu)) if ao != ag]
    return dict(anchors_oracle=a_o, anchors_gpu=list(t_gpu), moved=moved, path_cost=cost_oo,
                path_margin=cost_og - cost_oo, perturbation=pert, x_spread=float(x_o.std()))
