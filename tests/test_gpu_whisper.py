"""Model-level parity: the HIP Whisper path (libwdr through the C ABI) against the CPU
oracle (numpy restatement of the ggml graph + whisper_full loop + reference glue) on the
same synthetic weights and inputs.

Tolerances: normalised log-mel |err| <= 2e-3 (f32 DFT vs double FFT); encoder output and
logits compared relative to their spread (f16 operands, f32 accumulation on both sides,
different summation order); token ids / text identical; DTW anchors within 2 cs;
word times within 20 ms (the north-star bar)."""
import numpy as np
import pytest

import wdr
from oracle.mel import log_mel, pcm_i16_to_f32
from oracle.model import DecoderState, Whisper
from oracle.pipeline import SpeechSegment as OSeg
from oracle.pipeline import run_transcription_pipeline
from oracle.vocab import Vocab
from oracle.weights import hparams_for, synth_weights
from oracle.whisper_full import FullParams, WhisperState
from wdr.synth import synth_speech

pytestmark = pytest.mark.gpu

EMB_STD = 0.5
SYN = wdr.Synthetic(weight_std=0.02, emb_std=EMB_STD, force_len_rate=3.3, disable_fallback=True)


@pytest.fixture(scope="module", params=["tiny-test", "tiny-test-ml"])
def model(request):
    name = request.param
    ctx = wdr.WhisperContext(name, synthetic=SYN)
    hp = hparams_for(name)
    W = synth_weights(hp, std=0.02, emb_std=EMB_STD)
    return name, ctx, hp, W


@pytest.fixture(scope="module")
def audio():
    pcm, spurts = synth_speech(40.0, seed=0)
    return pcm, spurts


def test_log_mel_window_matches_oracle(model, audio):
    name, ctx, hp, W = model
    pcm, spurts = audio
    for a, b, _ in spurts[:3]:
        x = pcm_i16_to_f32(pcm[int(a * 16000):int(b * 16000)])
        got = ctx.log_mel_window(x, 0)
        ref = log_mel(x, hp.n_mels)[:, :3000]
        assert np.abs(got - ref).max() < 2e-3
    x = pcm_i16_to_f32(pcm[:16000 * 35])            # > 30 s: second window
    got = ctx.log_mel_window(x, 3000)
    ref = log_mel(x, hp.n_mels)[:, 3000:6000]
    assert np.abs(got - ref).max() < 2e-3


def test_encoder_matches_oracle(model):
    name, ctx, hp, W = model
    rng = np.random.default_rng(11)
    mel = (rng.standard_normal((hp.n_mels, 3000)) * 0.4).astype(np.float32)
    got = ctx.encode(mel)
    ref = Whisper(hp, W).encode(mel)
    err = np.abs(got - ref)
    assert err.max() < 5e-2 and err.mean() < 4e-3, (err.max(), err.mean())


def test_decoder_logits_and_capture_match_oracle(model):
    name, ctx, hp, W = model
    rng = np.random.default_rng(12)
    mel = (rng.standard_normal((hp.n_mels, 3000)) * 0.4).astype(np.float32)
    ctx.encode(mel)
    m = Whisper(hp, W)
    cross = m.cross_kv(m.encode(mel))
    v = Vocab(hp.n_vocab)
    for toks in ([v.sot], [v.sot, v.beg, 1234, 40000, 77], list(rng.integers(0, 50000, 20))):
        got = ctx.decode(toks)
        ref = DecoderState(m).forward(list(toks), cross)
        scale = ref.std()
        assert np.abs(got - ref).max() < 0.02 * scale + 0.02, (np.abs(got - ref).max(), scale)
        assert int(np.argmax(got)) == int(np.argmax(ref))
    toks = [v.sot, v.not_] + list(rng.integers(0, 50000, 12)) + [v.eot]
    from oracle.whisper_full import aheads_for_model_name
    ah = aheads_for_model_name(name)
    cap = ctx.capture(toks, len(ah))
    _, qk = DecoderState(m).forward(toks, cross, want_logits=None, aheads=ah)
    assert np.abs(cap - qk).max() < 2e-3
    np.testing.assert_allclose(cap.sum(-1), 1.0, atol=1e-3)


def _oracle_state(name, hp, W):
    return WhisperState(Whisper(hp, W), Vocab(hp.n_vocab), name)


def _params(lang="auto"):
    return FullParams(strategy="greedy", language=lang, force_len_rate=3.3, logprob_thold=-np.inf,
                      entropy_thold=-1.0)


@pytest.mark.parametrize("lang,strategy,temp", [("auto", "greedy", None), ("en", "greedy", None),
                                                ("en", "beam_search", None), ("auto", "beam_search", None),
                                                ("en", "greedy", 0.4), ("auto", "beam_search", 0.6)])
def test_state_full_matches_oracle(model, audio, lang, strategy, temp):
    """whisper_full_with_state: greedy, beam search (5 beams, whisper.cpp's default strategy in
    the reference, src/transcribe.rs:25-33) and the t > 0 sampling decoders (best_of 5,
    std::discrete_distribution + std::mt19937 per decoder)."""
    name, ctx, hp, W = model
    pcm, spurts = audio
    st = _oracle_state(name, hp, W)
    opts = wdr.TranscribeOptions(lang=lang, advanced=wdr.AdvancedTranscribe(sampling_strategy=strategy,
                                                                            temperature=temp))
    prompt = None
    for a, b, _ in spurts[:3]:
        x = pcm_i16_to_f32(pcm[int(a * 16000):int(b * 16000)])
        got, lang_id = ctx.state_full(x, opts, initial_prompt=prompt)
        p = _params(lang)
        p.strategy = "greedy" if strategy == "greedy" else "beam"
        if temp is not None:
            p.temperature = temp
        p.initial_prompt = prompt
        st.full(x, p)
        ref = st.result_all
        assert len(got) == len(ref)
        for g, r in zip(got, ref):
            assert [t["id"] for t in g["tokens"]] == [t.id for t in r.tokens]
            assert g["text"] == r.text
            assert (g["t0"], g["t1"]) == (r.t0, r.t1)
            for tg, tr in zip(g["tokens"], r.tokens):
                assert abs(tg["t_dtw"] - tr.t_dtw) <= 2, (tg, tr)
                assert abs(tg["t0"] - tr.t0) <= 2 and abs(tg["t1"] - tr.t1) <= 2, (tg, tr)
                assert abs(tg["p"] - tr.p) < 1e-3
        if lang == "auto":
            assert lang_id == st.lang_id
        prompt = ref[-1].text.lstrip() if ref else prompt


@pytest.mark.parametrize("translate", [False, True])
def test_pipeline_matches_oracle_glue(model, audio, translate):
    """run_transcription_pipeline: prompt chain, offsets, overlap clipping, callbacks order;
    translate: whisper_to_english (translate task token, src/transcribe.rs:54-55) with the
    interpolated word times of src/transcribe.rs:171-203."""
    name, ctx, hp, W = model
    pcm, spurts = audio
    segs = [wdr.SpeechSegment(a, b, pcm[int(a * 16000):int(b * 16000)]) for a, b, _ in spurts[:4]]
    events = []
    cb = wdr.Callbacks(progress=lambda p, t, l: events.append(("p", p, int(t), l)),
                       new_segment_callback=lambda s: events.append(("s", s.text)))
    opts = wdr.TranscribeOptions(lang="auto", offset=1.5, whisper_to_english=translate,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got, lang = ctx.run_pipeline(segs, opts, cb)
    st = _oracle_state(name, hp, W)
    ref, rlang = run_transcription_pipeline(st, [OSeg(s.start, s.end, s.samples) for s in segs],
                                            dict(lang="auto", offset=1.5, whisper_to_english=translate,
                                                 advanced=dict(sampling_strategy="greedy"),
                                                 synthetic=dict(force_len_rate=3.3, logprob_thold=-np.inf,
                                                                entropy_thold=-1.0)))
    assert lang == rlang
    assert [s.text for s in got] == [s.text for s in ref]
    for g, r in zip(got, ref):
        assert abs(g.start - r.start) <= 0.02 and abs(g.end - r.end) <= 0.02
        assert len(g.words) == len(r.words)
        for wg, wr in zip(g.words, r.words):
            assert wg.text == wr.text
            assert abs(wg.start - wr.start) <= 0.02 and abs(wg.end - wr.end) <= 0.02
    kinds = [e[0] for e in events]
    assert kinds == ["s", "p"] * len(got)
    assert [e[1] for e in events if e[0] == "p"] == [int((i + 1) / 4 * 100) for i in range(4)][:len(got)]
    assert all(e[3] == "Transcribing audio" and e[2] == 1 for e in events if e[0] == "p")


def test_engine_transcribe_audio_with_vad(tmp_path):
    """Engine::transcribe_audio with enable_vad: WAV -> GPU Silero VAD -> merged segments ->
    pipeline (src/engine.rs:123-139, 169-178) equals the pieces called one by one."""
    from oracle.pipeline import write_wav
    pcm, _ = synth_speech(25.0, seed=4)
    path = str(tmp_path / "a.wav")
    write_wav(path, pcm)
    eng = wdr.Engine(wdr.EngineConfig(), synthetic=SYN)
    opts = wdr.TranscribeOptions(model="tiny-test", lang="en", enable_vad=True,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got = eng.transcribe_audio(path, opts)
    mask, vsegs = wdr.Vad().get_segments(pcm)
    ctx = wdr.WhisperContext("tiny-test", synthetic=SYN)
    want, lang = ctx.run_pipeline(vsegs, opts)
    want = wdr.process_segments(want, lang or "en", None, mask)   # src/engine.rs:192-199
    assert len(vsegs) > 0
    assert [(s.text, round(s.start, 6), round(s.end, 6)) for s in got] == \
        [(s.text, round(s.start, 6), round(s.end, 6)) for s in want]


def _perturb_ln(W):
    """LayerNorm gamma/beta away from 1/0 (synthetic mode has no LN tensors to read), so a
    context that ignored the file's LN tensors would not match."""
    rng = np.random.default_rng(5)
    for k in list(W):
        if k.endswith("ln.weight") or k.endswith("_ln.weight") or k.endswith("ln_post.weight"):
            W[k] = (1.0 + 0.1 * rng.standard_normal(W[k].shape)).astype(np.float32)
        elif k.endswith("ln.bias") or k.endswith("_ln.bias") or k.endswith("ln_post.bias"):
            W[k] = (0.05 * rng.standard_normal(W[k].shape)).astype(np.float32)


@pytest.fixture(scope="module")
def ggml_model(tmp_path_factory):
    from tests.ggml_writer import write_ggml
    d = tmp_path_factory.mktemp("ggml")
    path = str(d / "ggml-tiny-test.bin")
    hp, _, _, W = write_ggml(path, "tiny-test", std=0.02, emb_std=EMB_STD, mutate=_perturb_ln)
    return path, hp, W


def test_ggml_file_context_matches_oracle(ggml_model, audio):
    """wdr_context_create(model_path=<whisper.cpp ggml file>): weights (f16 matrices, f32
    biases / LN / positional tables), mel filters and vocabulary come from the file
    (src/transcribe.rs:154); encoder and full decode match the oracle on the same weights."""
    path, hp, W = ggml_model
    ctx = wdr.WhisperContext("tiny-test", model_path=path, synthetic=SYN)
    assert ctx.hparams["n_vocab"] == hp.n_vocab and ctx.hparams["n_mels"] == hp.n_mels
    rng = np.random.default_rng(11)
    mel = (rng.standard_normal((hp.n_mels, 3000)) * 0.4).astype(np.float32)
    got = ctx.encode(mel)
    ref = Whisper(hp, W).encode(mel)
    err = np.abs(got - ref)
    assert err.max() < 5e-2 and err.mean() < 4e-3, (err.max(), err.mean())
    syn_out = wdr.WhisperContext("tiny-test", synthetic=SYN).encode(mel)
    assert np.abs(syn_out - ref).mean() > 10 * err.mean()   # the file's LN tensors were used
    pcm, spurts = audio
    st = _oracle_state("tiny-test", hp, W)
    for a, b, _ in spurts[:2]:
        x = pcm_i16_to_f32(pcm[int(a * 16000):int(b * 16000)])
        g, lang_id = ctx.state_full(x, wdr.TranscribeOptions(
            lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy")))
        st.full(x, _params("auto"))
        assert [[t["id"] for t in s["tokens"]] for s in g] == [[t.id for t in r.tokens] for r in st.result_all]
        assert [s["text"] for s in g] == [r.text for r in st.result_all]
        assert lang_id == st.lang_id


def test_engine_loads_cached_ggml_file(ggml_model, tmp_path):
    """Engine::transcribe_audio resolves ggml-<model>.bin in the hf-hub cache layout
    (<cache>/models--ggerganov--whisper.cpp/snapshots/<rev>/, src/model_manager.rs:661-681)
    and transcribes with the file's weights: same output as a context made from that file."""
    import shutil
    from oracle.pipeline import write_wav
    path, hp, W = ggml_model
    snap = tmp_path / "cache" / "models--ggerganov--whisper.cpp" / "snapshots" / "rev0"
    snap.mkdir(parents=True)
    shutil.copy(path, snap / "ggml-tiny-test.bin")
    pcm, _ = synth_speech(25.0, seed=4)
    wav = str(tmp_path / "a.wav")
    write_wav(wav, pcm)
    eng = wdr.Engine(wdr.EngineConfig(cache_dir=str(tmp_path / "cache")), synthetic=SYN)
    opts = wdr.TranscribeOptions(model="tiny-test", lang="en", enable_vad=True,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got = eng.transcribe_audio(wav, opts)
    mask, vsegs = wdr.Vad().get_segments(pcm)
    ctx = wdr.WhisperContext("tiny-test", model_path=path, synthetic=SYN)
    want, lang = ctx.run_pipeline(vsegs, opts)
    want = wdr.process_segments(want, lang or "en", None, mask)
    assert len(got) > 0
    assert [(s.text, round(s.start, 6), round(s.end, 6)) for s in got] == \
        [(s.text, round(s.start, 6), round(s.end, 6)) for s in want]


@pytest.mark.parametrize("translate", [False, True])
def test_engine_whole_file_path(tmp_path, translate):
    """Engine::transcribe_audio with neither VAD nor diarization: the whole file is one speech
    segment (src/engine.rs:141-147), then process_segments without a VAD mask
    (src/engine.rs:179-199); with whisper_to_english the words are interpolated."""
    from oracle.pipeline import write_wav
    pcm, _ = synth_speech(20.0, seed=7)
    path = str(tmp_path / "w.wav")
    write_wav(path, pcm)
    eng = wdr.Engine(wdr.EngineConfig(), synthetic=SYN)
    opts = wdr.TranscribeOptions(model="tiny-test-ml", lang="auto", whisper_to_english=translate, enable_vad=False,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got = eng.transcribe_audio(path, opts)
    ctx = wdr.WhisperContext("tiny-test-ml", synthetic=SYN)
    want, lang = ctx.run_pipeline([wdr.SpeechSegment(0.0, len(pcm) / 16000.0, pcm)], opts)
    want = wdr.process_segments(want, lang or "auto", None, None)
    assert len(got) > 0
    assert [(s.text, round(s.start, 6), round(s.end, 6)) for s in got] == \
        [(s.text, round(s.start, 6), round(s.end, 6)) for s in want]
    assert [[(w.text, round(w.start, 6), round(w.end, 6)) for w in s.words] for s in got] == \
        [[(w.text, round(w.start, 6), round(w.end, 6)) for w in s.words] for s in want]


@pytest.mark.parametrize("chains", [1, 4])
def test_cancellation_through_c_abi(chains):
    """Callbacks::is_cancelled (src/engine.rs:35-40) wired to whisper.cpp's abort callback
    (src/transcribe.rs:348-350): once it returns true the run stops with "failed to transcribe"
    -- polled before each segment (one chain) or by the calling thread while the decode chains
    run (multi-chain: chains stop at their next segment).  The context is reusable afterwards:
    the next uncancelled run equals a fresh one (no stale DTW job, batcher seat or slot left)."""
    name = "tiny-test"
    ctx = wdr.WhisperContext(name, synthetic=SYN)
    ctx.set_chains(chains)
    pcm, spurts = synth_speech(40.0, seed=0)
    segs = [wdr.SpeechSegment(a, b, pcm[int(a * 16000):int(b * 16000)]) for a, b, _ in spurts]
    assert len(segs) >= 6
    opts = wdr.TranscribeOptions(lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    ref, _ = ctx.run_pipeline(segs, opts)
    seen = []
    if chains == 1:
        cb = wdr.Callbacks(new_segment_callback=lambda s: seen.append(s.text), is_cancelled=lambda: len(seen) >= 2)
    else:
        cb = wdr.Callbacks(new_segment_callback=lambda s: seen.append(s.text), is_cancelled=lambda: True)
    with pytest.raises(wdr.WdrError, match="failed to transcribe"):
        ctx.run_pipeline(segs, opts, cb)
    assert len(seen) < len(ref)
    if chains == 1:
        assert seen == [s.text for s in ref[:len(seen)]] and len(seen) >= 2
    again, _ = ctx.run_pipeline(segs, opts)
    assert [(s.text, s.start, s.end) for s in again] == [(s.text, s.start, s.end) for s in ref]
    ctx.close()
