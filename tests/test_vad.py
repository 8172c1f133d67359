"""Silero VAD: the HIP forward and the C++ segment state machine
against oracle/vad.py (parity unpinned against whisper.cpp itself -- see oracle/vad.py)."""
import os
import sys

import numpy as np
import pytest

import wdr
from oracle import vad as ovad
from oracle.pipeline import vad_merge

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "whisper-diarize-rs_amd"))
from wdr.synth import synth_speech  # noqa: E402


def _prob_tracks(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 3000))
    # piecewise-constant speech / silence runs with noise, crossing 0.5 / 0.35 often
    out, t = [], 0
    while t < n:
        run = int(rng.integers(1, 80))
        level = rng.choice([0.9, 0.6, 0.45, 0.3, 0.1])
        out.extend(np.clip(level + 0.08 * rng.standard_normal(run), 0, 1))
        t += run
    return np.asarray(out[:n], np.float32)


@pytest.mark.parametrize("seed", range(12))
def test_segments_from_probs_matches_oracle(seed):
    p = _prob_tracks(seed)
    got = wdr.vad_segments_from_probs(p)
    want = ovad.segments_from_probs(p)
    assert got == want


def test_segments_from_probs_edges():
    assert wdr.vad_segments_from_probs(np.zeros(0, np.float32)) == []
    assert wdr.vad_segments_from_probs(np.ones(1, np.float32)) == ovad.segments_from_probs(np.ones(1))
    for p in (np.ones(200, np.float32), np.zeros(200, np.float32), np.r_[np.ones(100), np.zeros(3), np.ones(100)],
              np.r_[np.zeros(5), np.ones(8), np.zeros(50)], np.full(100, 0.5, np.float32),
              np.full(100, 0.35, np.float32)):
        p = np.asarray(p, np.float32)
        assert wdr.vad_segments_from_probs(p) == ovad.segments_from_probs(p)


def test_oracle_chunking_reflect_pad():
    x = np.arange(1100, dtype=np.float32)
    fr = ovad.chunk_frames(x)
    assert fr.shape == (3, 640)
    np.testing.assert_array_equal(fr[0, :64], np.arange(64, 0, -1))
    np.testing.assert_array_equal(fr[0, 64:576], np.arange(512))
    np.testing.assert_array_equal(fr[0, 576:], np.arange(510, 446, -1))
    # last chunk: 76 real samples, zero fill
    assert fr[2, 64 + 76:576].max() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [300, 512, 513, 16000 * 20 + 77])
def test_vad_probs_match_oracle(n):
    pcm, _ = synth_speech(n / 16000.0 + 0.01, seed=3, n_speakers=1)
    pcm = pcm[:n]
    v = wdr.Vad()
    got = v.probs(pcm)
    want = ovad.probs(pcm.astype(np.float32) / np.float32(32768.0), ovad.vad_weights())
    assert got.shape == want.shape
    # f16-rounded operands, f32 sums in a different order; the recurrent state enters W_hh as
    # f16, so a last-bit difference can flip one f16 rounding of h (2^-11 relative): bounded
    # (the LSTM is contractive), not accumulating
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-3)
    assert np.abs(got - want).mean() < 2e-4


@pytest.mark.gpu
def test_vad_get_segments_matches_reference_glue():
    pcm, _ = synth_speech(45.0, seed=1, n_speakers=2)
    v = wdr.Vad()
    p = v.probs(pcm)
    mask, segs = v.get_segments(pcm)
    # the oracle state machine + reference merge on the GPU's probabilities
    mask_o, segs_o = vad_merge(ovad.segments_from_probs(p), pcm)
    assert mask == mask_o
    assert [(s.start, s.end) for s in segs] == [(s.start, s.end) for s in segs_o]
    for a, b in zip(segs, segs_o):
        np.testing.assert_array_equal(a.samples, b.samples)
    assert v.last_us_per_step > 0


@pytest.mark.gpu
def test_vad_empty_input():
    v = wdr.Vad()
    assert v.probs(np.zeros(0, np.int16)).size == 0
    assert v.get_segments(np.zeros(0, np.int16)) == ([], [])
