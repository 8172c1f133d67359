"""Pin the CPU oracle against the golden fixtures (tests/golden/make_golden.py).

These are CPU tests: the oracle must agree with the third-party golden vectors
before it is trusted as the parity checker for the HIP path.
"""
import os

import numpy as np

from conftest import GOLDEN
from oracle import dtw as odtw
from oracle import mel as omel
from oracle.model import Whisper, gelu_erf
from oracle.model import DecoderState
from oracle.weights import hparams_for, synth_weights


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def test_mel_filters_match_transformers():
    g = _load("mel_filters.npz")
    for n in (80, 128):
        f = omel.mel_filters(n)
        assert f.shape == (n, 201)
        np.testing.assert_allclose(f, g["f%d" % n], rtol=1e-5, atol=1e-7)


def test_power_spectrum_matches_transformers():
    g = _load("power_spec.npz")
    x, ref = g["x"], g["power"]
    hann = omel.hann_periodic().astype(np.float64)
    for i in range(ref.shape[0]):
        fr = x[i * 160:i * 160 + 400].astype(np.float64) * hann
        p = np.abs(np.fft.rfft(fr)) ** 2
        np.testing.assert_allclose(p, ref[i], rtol=1e-5, atol=1e-9)


def test_dtw_matches_transformers_including_ties():
    g = _load("dtw_cases.npz")
    keys = sorted(int(k[1:]) for k in g.files if k.startswith("x"))
    assert len(keys) >= 8
    for k in keys:
        x = g["x%d" % k]
        ti, tj = odtw.dtw(x)
        np.testing.assert_array_equal(ti, g["ti%d" % k])
        np.testing.assert_array_equal(tj, g["tj%d" % k])
        # the anti-diagonal formulation is identical to the j-outer/i-inner loop
        if x.size <= 2000:
            c1, t1 = odtw.dtw_cost_matrix(x)
            c2, t2 = odtw.dtw_cost_matrix_fast(x)
            np.testing.assert_array_equal(t1, t2)
            np.testing.assert_array_equal(c1, c2)


def test_median_filter_matches_transformers():
    g = _load("medfilt.npz")
    np.testing.assert_array_equal(odtw.median_filter(g["x"], 7), g["y"])


def test_whisper_f32_graph_matches_transformers():
    g = _load("whisper_tiny.npz")
    hp = hparams_for("tiny-test")
    W = synth_weights(hp, std=0.02, emb_std=0.2)
    m = Whisper(hp, W, f16in=False, conv_act=gelu_erf)
    enc = m.encode(g["mel"])
    np.testing.assert_allclose(enc[::25], g["enc_rows"], rtol=2e-3, atol=2e-3)
    cross = m.cross_kv(enc)
    st = DecoderState(m)
    logits, qk = st.forward(list(g["tokens"]), cross, want_logits="all", aheads=[(1, 0), (1, 1)])
    np.testing.assert_allclose(logits[-1], g["logits_last"], rtol=0, atol=5e-3)
    assert (np.argsort(-logits, axis=1)[:, :5] == g["logits_top"][:, :5]).mean() > 0.95
    np.testing.assert_allclose(qk, g["cross_last"], rtol=0, atol=1e-5)


def test_f16_rounding_graph_is_close_to_f32_graph():
    """The ggml-rounding oracle (f16 activations into matmuls) stays close to the f32 graph."""
    hp = hparams_for("tiny-test")
    W = synth_weights(hp, std=0.02, emb_std=0.2)
    g = _load("whisper_tiny.npz")
    a = Whisper(hp, W, f16in=False).encode(g["mel"])
    b = Whisper(hp, W, f16in=True).encode(g["mel"])
    assert np.abs(a - b).max() < 5e-2
    assert np.abs(a - b).mean() < 5e-3


def test_signal_energy_matches_naive_loop():
    rng = np.random.default_rng(0)
    x = rng.standard_normal(500).astype(np.float32)
    e = omel.signal_energy(x)
    for i in (0, 1, 31, 32, 250, 467, 499):
        s = np.float32(0)
        for j in range(-32, 33):
            if 0 <= i + j < 500:
                s = np.float32(s + np.float32(abs(x[i + j])))
        assert e[i] == np.float32(s / np.float32(65))


def test_log_mel_shapes_and_pad_value():
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(16000 * 3) * 0.1).astype(np.float32)
    m = omel.log_mel(x, 80)
    n_len, n_len_org = omel.mel_lengths(x.size)
    assert m.shape == (80, n_len) and n_len == (x.size + 480000) // 160
    assert n_len_org == 1 + (x.size + 200 - 400) // 160
    # the zero-padded tail sits at the clamp floor max(-10, max-8), normalised
    tail = m[:, -10:]
    assert np.allclose(tail, tail[0, 0])
    assert m.max() == np.float32((m.max() * 4 - 4 + 4) / 4)


def test_oracle_beam_search_with_one_beam_is_greedy():
    """Beam search with K = 1 reduces to greedy (top-1 = argmax, ties by lower id)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "whisper-diarize-rs_amd"))
    from oracle.model import Whisper
    from oracle.vocab import Vocab
    from oracle.weights import hparams_for, synth_weights
    from oracle.whisper_full import FullParams, WhisperState
    from oracle.mel import pcm_i16_to_f32
    from wdr.synth import synth_speech
    hp = hparams_for("tiny-test")
    W = synth_weights(hp, std=0.02, emb_std=0.5)
    pcm, sp = synth_speech(12.0, seed=0)
    x = pcm_i16_to_f32(pcm[int(sp[0][0] * 16000):int(sp[0][1] * 16000)])
    out = []
    for strat, k in (("greedy", 5), ("beam", 1), ("beam", 3)):
        st = WhisperState(Whisper(hp, W), Vocab(hp.n_vocab), "tiny-test")
        p = FullParams(strategy=strat, beam_size=k, language="en", force_len_rate=3.3,
                       logprob_thold=-np.inf, entropy_thold=-1.0)
        st.full(x, p)
        out.append([t.id for r in st.result_all for t in r.tokens])
    assert out[0] == out[1]
    assert len(out[2]) == len(out[0])
