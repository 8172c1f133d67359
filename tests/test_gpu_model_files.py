"""VAD and diarization on the GPU with weights read from model files:
the Silero ggml file and the segmentation-3.0 / CAM++ ONNX graphs written from mutated oracle
weights (tests/model_writers.py) drive libwdr's models, which must match the oracle on the
file's weights (tolerances as tests/test_vad.py and tests/test_gpu_diarize.py) and differ
from the synthetic-weight models.  The Engine resolves the files from its cache directory
like the reference's model manager (src/model_manager.rs:303-351) and uses them."""
import numpy as np
import pytest

import wdr
from oracle import diarize as D
from oracle import vad as V
from oracle.pipeline import write_wav
from tests.model_writers import write_campplus_onnx, write_segmentation_onnx, write_silero_ggml
from wdr.synth import synth_speech

pytestmark = pytest.mark.gpu
SYN = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)


def test_vad_from_ggml_file(tmp_path):
    p = str(tmp_path / "ggml-silero-v5.1.2.bin")
    W = write_silero_ggml(p)
    pcm, _ = synth_speech(12.0, seed=5)
    got = wdr.Vad(model_path=p).probs(pcm)
    want = V.probs(pcm.astype(np.float32) / np.float32(32768.0), W)
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-3)
    assert np.abs(got - want).mean() < 2e-4
    syn = wdr.Vad().probs(pcm)
    assert np.abs(syn - want).mean() > 10 * np.abs(got - want).mean()


@pytest.mark.parametrize("gemm", [False, True])
def test_segmentation_from_onnx_file(tmp_path, gemm):
    p = str(tmp_path / "segmentation-3.0.onnx")
    W = write_segmentation_onnx(p, gemm=gemm)
    pcm, _ = synth_speech(14.0, seed=6, n_speakers=2)
    dz = wdr.Diarizer(segment_model_path=p)
    cls, lp = dz.frame_classes(pcm, logprobs=True)
    padded = np.zeros(cls.shape[0] * 160000, np.float32)
    padded[:pcm.size] = pcm
    for w in range(cls.shape[0]):
        ref = D.seg_window(padded[w * 160000:(w + 1) * 160000], W)
        np.testing.assert_allclose(lp[w], ref, rtol=0, atol=1e-3)
        srt = np.sort(ref, 1)
        clear = (srt[:, -1] - srt[:, -2]) > 1e-3
        assert (cls[w][clear] == np.array([D.last_argmax(r) for r in ref])[clear]).all()
    _, lp_syn = wdr.Diarizer().frame_classes(pcm, logprobs=True)
    assert np.abs(lp_syn - lp).max() > 0.1


@pytest.mark.parametrize("fused", [False, True])
def test_campplus_from_onnx_file(tmp_path, fused):
    p = str(tmp_path / "wespeaker_en_voxceleb_CAM++.onnx")
    W = write_campplus_onnx(p, fused=fused)
    pcm, _ = synth_speech(9.0, seed=7)
    dz = wdr.Diarizer(embedding_model_path=p)
    for x in (pcm[:16000 * 3], pcm[3000:3000 + 16000 * 7 + 11]):
        e = dz.embedding(x)
        r = D.campplus(D.compute_feats(x), W)
        np.testing.assert_allclose(e, r, rtol=1e-3, atol=1e-3)
        assert D.EmbeddingManager.cosine(e, r) > 0.9999
        assert D.EmbeddingManager.cosine(wdr.Diarizer().embedding(x), r) < 0.999


def test_engine_uses_cached_model_files(tmp_path):
    """Engine::transcribe_audio (src/engine.rs:89-139): with the VAD / diarization model files
    in the cache dir (ggml-org/whisper-vad hf-hub layout for Silero, the ONNX files at the cache
    root) the Engine loads them -- and without them, outside synthetic mode, it fails."""
    cache = tmp_path / "cache"
    snap = cache / "models--ggml-org--whisper-vad" / "snapshots" / "r0"
    snap.mkdir(parents=True)
    vad_path = str(snap / "ggml-silero-v5.1.2.bin")
    write_silero_ggml(vad_path)
    seg_path, emb_path = str(cache / "segmentation-3.0.onnx"), str(cache / "wespeaker_en_voxceleb_CAM++.onnx")
    write_segmentation_onnx(seg_path, seed=None)   # the synthetic calibration: frames split speech / silence
    write_campplus_onnx(emb_path)
    pcm, _ = synth_speech(25.0, seed=8, n_speakers=2)
    wav = str(tmp_path / "a.wav")
    write_wav(wav, pcm)
    eng = wdr.Engine(wdr.EngineConfig(cache_dir=str(cache)), synthetic=SYN)
    ctx = wdr.WhisperContext("tiny-test", synthetic=SYN)
    # VAD branch
    opts = wdr.TranscribeOptions(model="tiny-test", lang="en", enable_vad=True,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got = eng.transcribe_audio(wav, opts)
    mask, vsegs = wdr.Vad(model_path=vad_path).get_segments(pcm)
    want, lang = ctx.run_pipeline(vsegs, opts)
    want = wdr.process_segments(want, lang or "en", None, mask)
    assert [(s.text, round(s.start, 6)) for s in got] == [(s.text, round(s.start, 6)) for s in want]
    # diarize branch
    opts = wdr.TranscribeOptions(model="tiny-test", lang="en", enable_diarize=True,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got = eng.transcribe_audio(wav, opts)
    dsegs = wdr.Diarizer(segment_model_path=seg_path).get_segments(pcm)
    assert len(dsegs) > 0
    want, lang = ctx.run_pipeline(dsegs, opts, diarize_options=wdr.DiarizeOptions.from_options(opts, seg_path, emb_path))
    want = wdr.process_segments(want, lang or "en")
    assert len(got) > 0
    assert [(s.text, s.speaker_id, round(s.start, 6)) for s in got] == \
        [(s.text, s.speaker_id, round(s.start, 6)) for s in want]
    # no files and no synthetic mode: the reference would try to download; offline it fails
    eng2 = wdr.Engine(wdr.EngineConfig(cache_dir=str(tmp_path / "empty")), synthetic=None)
    with pytest.raises(wdr.WdrError, match="doesn't exist"):
        eng2.transcribe_audio(wav, opts)
