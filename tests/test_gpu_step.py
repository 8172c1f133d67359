"""The decoder-rows contract (csrc/rows.h) on the GPU: a decode step is a row like any other.

A prefill of n tokens followed by nothing, and a prefill of n-1 tokens followed by ONE decode
step of the n-th, compute the n-th row with the same kernels: bit-identical logits while the
prefill's rows form a VALU cross-attention group (n <= 8); above that the prefill's
cross-attention runs on the MFMA tile kernel (a different summation order), so the logits are
compared relative to their spread (|err| <= 0.01 * std + 0.01, same argmax).  The step is also
checked against the CPU oracle.  Widths: tiny-test (d 128), base.en (d 512), large-v3 (d 1280,
20 heads, 32 layers)."""
import numpy as np
import pytest

import wdr
from oracle.model import DecoderState, Whisper
from oracle.vocab import Vocab
from oracle.weights import hparams_for, synth_weights

pytestmark = pytest.mark.gpu


def _close(a, b):
    scale = float(b.std())
    err = float(np.abs(a - b).max())
    assert err <= 0.01 * scale + 0.01, (err, scale)


@pytest.mark.parametrize("name", ["tiny-test", "base.en", "large-v3"])
def test_step_row_equals_prefill_row(name):
    ctx = wdr.WhisperContext(name, synthetic=wdr.Synthetic(weight_std=0.02, emb_std=0.5))
    hp = ctx.hparams
    rng = np.random.default_rng(3)
    mel = (rng.standard_normal((hp["n_mels"], 3000)) * 0.4).astype(np.float32)
    ctx.encode(mel)
    v = Vocab(hp["n_vocab"])
    seqs = [[v.sot, v.beg], [v.sot, v.beg, 1234, 40000, 77], list(rng.integers(0, 50000, 8)),
            list(rng.integers(0, 50000, 37)), list(rng.integers(0, 50000, 300)),
            list(rng.integers(0, 50000, 448))]
    for toks in seqs:
        step = ctx.step(toks)
        pre = ctx.decode(toks)
        assert np.isfinite(step).all()
        if len(toks) <= 8:
            np.testing.assert_array_equal(step, pre)
        else:
            _close(step, pre)
            assert int(np.argmax(step)) == int(np.argmax(pre))
    # back-to-back: the same inputs give the same bits
    toks = [v.sot, v.beg, 500, 600]
    first = ctx.step(toks)
    for _ in range(10):
        np.testing.assert_array_equal(ctx.step(toks), first)
    ctx.close()


def test_step_matches_oracle():
    name = "tiny-test"
    ctx = wdr.WhisperContext(name, synthetic=wdr.Synthetic(weight_std=0.02, emb_std=0.5))
    hp = hparams_for(name)
    W = synth_weights(hp, std=0.02, emb_std=0.5)
    rng = np.random.default_rng(12)
    mel = (rng.standard_normal((hp.n_mels, 3000)) * 0.4).astype(np.float32)
    ctx.encode(mel)
    m = Whisper(hp, W)
    cross = m.cross_kv(m.encode(mel))
    v = Vocab(hp.n_vocab)
    for toks in ([v.sot, v.beg, 1234, 40000, 77], list(rng.integers(0, 50000, 20))):
        got = ctx.step(toks)
        ref = DecoderState(m).forward(list(toks), cross)
        scale = ref.std()
        assert np.abs(got - ref).max() < 0.02 * scale + 0.02, (np.abs(got - ref).max(), scale)
        assert int(np.argmax(got)) == int(np.argmax(ref))
    ctx.close()
