"""Diarization rows a16-a19 on the GPU (libwdr through the C ABI) against oracle/diarize.py.

Tolerances: both sides are f32 (the reference runs ONNX Runtime f32); the GPU sums in a
different order (tiled GEMM, f32 DFT instead of a double FFT), so log-probabilities within
1e-3, fbank within 2e-3, embeddings within 1e-3 (cosine > 0.9999).  Frame classes must be
identical wherever the top-2 log-probability margin exceeds 1e-3; segment stitching is
compared exactly on the GPU's own classes."""
import numpy as np
import pytest

import wdr
from wdr import _lib as L
from oracle import diarize as D
from oracle.pipeline import write_wav
from wdr.synth import synth_speech

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dz():
    return wdr.Diarizer()


@pytest.fixture(scope="module")
def audio():
    pcm, spurts = synth_speech(27.0, seed=2, n_speakers=3)
    return pcm, spurts


def test_segmentation_logprobs_and_classes(dz, audio):
    pcm, _ = audio
    cls, lp = dz.frame_classes(pcm, logprobs=True)
    W = D.seg_weights()
    padded = np.zeros(cls.shape[0] * 160000, np.float32)
    padded[:pcm.size] = pcm
    for w in range(cls.shape[0]):
        ref = D.seg_window(padded[w * 160000:(w + 1) * 160000], W)
        np.testing.assert_allclose(lp[w], ref, rtol=0, atol=1e-3)
        srt = np.sort(ref, 1)
        clear = (srt[:, -1] - srt[:, -2]) > 1e-3
        want = np.array([D.last_argmax(r) for r in ref])
        assert (cls[w][clear] == want[clear]).all()


def test_get_segments_stitching(dz, audio):
    pcm, _ = audio
    cls = dz.frame_classes(pcm)
    segs = dz.get_segments(pcm)
    want = D.get_segments_from_argmax(pcm.size, cls)
    assert len(segs) == len(want) and len(want) > 0
    padded = np.zeros(cls.shape[0] * 160000, np.int16)
    padded[:pcm.size] = pcm
    for s, (a, b, si, ei) in zip(segs, want):
        assert s.start == a and s.end == b
        np.testing.assert_array_equal(s.samples, padded[si:ei])


@pytest.mark.parametrize("n", [399, 400, 16000, 59213, 16000 * 12 + 7])
def test_fbank_and_embedding(dz, audio, n):
    pcm, _ = audio
    x = pcm[1000:1000 + n]
    f = dz.fbank(x)
    ref = D.compute_feats(x)
    assert f.shape == ref.shape
    np.testing.assert_allclose(f, ref, rtol=0, atol=2e-3)
    e = dz.embedding(x)
    r = D.compute_embedding(x, D.cam_weights())
    if r is None:
        assert e is None
        return
    np.testing.assert_allclose(e, r, rtol=1e-3, atol=1e-3)   # NaN where the std of 1 frame is NaN (torch too)
    if np.isnan(r).any():
        return
    assert D.EmbeddingManager.cosine(e, r) > 0.9999
    assert dz.stats()[1] > 0


def test_embedding_batch_equals_single(dz, audio):
    """The pipeline's embedding worker runs CamModel::embed_batch over many utterances at once;
    per utterance it must be bit-identical to the one-utterance forward (ragged lengths, a
    too-short utterance with no frames, a 1-frame utterance)."""
    pcm, spurts = audio
    segs = [pcm[int(a * 16000):int(b * 16000)] for a, b, _ in spurts]
    segs = segs[:6] + [pcm[:399], pcm[5000:5400], pcm[7000:7000 + 16000 * 11 + 3]] + segs[6:9]
    got = dz.embedding_batch(segs)
    assert len(got) == len(segs)
    for x, g in zip(segs, got):
        e = dz.embedding(x)
        if e is None:
            assert g is None
            continue
        np.testing.assert_array_equal(g, e)
    assert dz.embedding_batch([]) == []


SYN = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)


def test_pipeline_assigns_speakers_like_the_reference_glue(dz, audio):
    pcm, spurts = audio
    segs = [wdr.SpeechSegment(a, b, pcm[int(a * 16000):int(b * 16000)]) for a, b, _ in spurts[:5]]
    ctx = wdr.WhisperContext("tiny-test", synthetic=SYN)
    for max_spk, thr in ((None, 0.5), (2, 0.9999)):
        opts = wdr.TranscribeOptions(lang="en", enable_diarize=True, max_speakers=max_spk,
                                     advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy", diarize_threshold=thr))
        got, _ = ctx.run_pipeline(segs, opts, diarize_options=wdr.DiarizeOptions.from_options(opts))
        plain, _ = ctx.run_pipeline(segs, wdr.TranscribeOptions(
            lang="en", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy")))
        assert [s.text for s in got] == [s.text for s in plain]
        mgr = D.EmbeddingManager(max_spk if max_spk else 2 ** 64 - 1)
        # one whisper segment per speech segment here (single_segment, < 30 s)
        want = [mgr.assign(dz.embedding(s.samples), thr) for s in segs][:len(got)]
        assert [s.speaker_id for s in got] == want


def test_engine_transcribe_audio_with_diarize(tmp_path, dz):
    pcm, _ = synth_speech(22.0, seed=6, n_speakers=2)
    path = str(tmp_path / "d.wav")
    write_wav(path, pcm)
    eng = wdr.Engine(wdr.EngineConfig(), synthetic=SYN)
    opts = wdr.TranscribeOptions(model="tiny-test", lang="en", enable_diarize=True,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got = eng.transcribe_audio(path, opts)
    segs = dz.get_segments(pcm)
    ctx = wdr.WhisperContext("tiny-test", synthetic=SYN)
    want, lang = ctx.run_pipeline(segs, opts, diarize_options=wdr.DiarizeOptions.from_options(opts))
    want = wdr.process_segments(want, lang or "en")   # no VAD mask on the diarize branch
    assert [(s.text, s.speaker_id, round(s.start, 6)) for s in got] == \
        [(s.text, s.speaker_id, round(s.start, 6)) for s in want]


def test_mfma_f32_gemm_equals_valu(dz, audio):
    """The segmentation / CAM++ contractions on v_mfma_f32_32x32x2_f32 (k_gemm32m, default) and on
    the VALU f32 kernel (wdr_dbg_set_gemm32(0)): both are one f32 fma per k in k order, so log-probabilities
    and embeddings must agree to f32 rounding of the epilogues (1e-5), and the frame classes
    exactly wherever the class margin exceeds 1e-4."""
    pcm, spurts = audio
    cls, lp = dz.frame_classes(pcm, logprobs=True)
    x = pcm[int(spurts[0][0] * 16000):int(spurts[0][1] * 16000)]
    e = dz.embedding(x)
    lib = L.load()
    L.check(lib.wdr_dbg_set_gemm32(0))
    try:
        cls0, lp0 = dz.frame_classes(pcm, logprobs=True)
        e0 = dz.embedding(x)
    finally:
        L.check(lib.wdr_dbg_set_gemm32(1))
    np.testing.assert_allclose(lp, lp0, rtol=0, atol=1e-5)
    srt = np.sort(lp0, -1)
    clear = (srt[..., -1] - srt[..., -2]) > 1e-4
    assert (cls[clear] == cls0[clear]).all()
    np.testing.assert_allclose(e, e0, rtol=1e-5, atol=1e-5)
