"""CPU-side tests: libwdr loads and exports the C ABI, and the host-only seams
(read_wav, the reference's VAD merge) match the oracle's restatement of the reference glue."""
import os
import struct

import numpy as np
import pytest

from oracle import pipeline as op
from wdr import _lib
import wdr


def test_library_exports_every_header_symbol(lib):
    syms = _lib.header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.wdr_abi_version() == 6


def _wav(path, samples, ch=1, rate=16000, bits=16, fmt=1):
    data = np.asarray(samples, np.int16).tobytes() if bits == 16 else bytes(len(samples))
    hdr = b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, fmt, ch, rate, rate * ch * bits // 8, ch * bits // 8, bits)
    hdr += b"data" + struct.pack("<I", len(data))
    with open(path, "wb") as f:
        f.write(hdr + data)


def test_read_wav_roundtrip_and_reference_errors(tmp_path):
    x = (np.random.default_rng(0).standard_normal(16000) * 3000).astype(np.int16)
    p = str(tmp_path / "a.wav")
    op.write_wav(p, x)
    np.testing.assert_array_equal(wdr.read_wav(p), x)
    np.testing.assert_array_equal(op.read_wav(p), x)
    cases = [
        (dict(ch=2), "expected mono audio file and found 2 channels!"),
        (dict(rate=44100), "expected 16KHz sample rate"),
        (dict(bits=8), "expected 16 bits per sample"),
        (dict(fmt=3), "expected integer sample format"),
    ]
    for kw, msg in cases:
        q = str(tmp_path / "b.wav")
        _wav(q, x[:100], **kw)
        with pytest.raises(wdr.WdrError, match=msg):
            wdr.read_wav(q)
        with pytest.raises(op.WavError, match=msg):
            op.read_wav(q)
    with pytest.raises(wdr.WdrError, match="failed to read file"):
        wdr.read_wav(str(tmp_path / "missing.wav"))


def test_transcribe_audio_missing_file_message():
    e = wdr.Engine(wdr.EngineConfig())
    with pytest.raises(wdr.WdrError, match="audio file doesn't exist"):
        e.transcribe_audio("/nonexistent/x.wav", wdr.TranscribeOptions())


def test_missing_whisper_model_fails_like_the_reference(tmp_path):
    """No ggml-<model>.bin in the cache and no explicit synthetic mode: transcribe_audio fails
    with the reference's "whisper file doesn't exist" (src/transcribe.rs:99-101) before touching
    the GPU -- it never falls back to random weights silently."""
    from oracle.pipeline import write_wav
    wav = str(tmp_path / "a.wav")
    write_wav(wav, np.zeros(16000, np.int16))
    e = wdr.Engine(wdr.EngineConfig(cache_dir=str(tmp_path / "empty_cache")))
    for model in ("base.en", "large-v3", "tiny-test"):
        with pytest.raises(wdr.WdrError, match="whisper file doesn't exist"):
            e.transcribe_audio(wav, wdr.TranscribeOptions(model=model, enable_vad=False))
    # create_context: a missing path, and no path without synthetic mode
    with pytest.raises(wdr.WdrError, match="whisper file doesn't exist"):
        wdr.WhisperContext("base.en", model_path=str(tmp_path / "ggml-base.en.bin"))
    with pytest.raises(wdr.WdrError, match="whisper file doesn't exist"):
        wdr.WhisperContext("base.en")


def test_missing_vad_and_diarize_model_files_fail(tmp_path):
    """A model path that does not exist is an error, never a silent synthetic fallback."""
    with pytest.raises(wdr.WdrError, match="VAD model file doesn't exist"):
        wdr.Vad(model_path=str(tmp_path / "ggml-silero-v5.1.2.bin"))
    with pytest.raises(wdr.WdrError, match="diarization model file doesn't exist"):
        wdr.Diarizer(segment_model_path=str(tmp_path / "segmentation-3.0.onnx"))
    with pytest.raises(wdr.WdrError, match="diarization model file doesn't exist"):
        wdr.Diarizer(embedding_model_path=str(tmp_path / "cam.onnx"))


def test_vad_merge_matches_reference_glue():
    rng = np.random.default_rng(3)
    samples = rng.integers(-3000, 3000, 16000 * 20).astype(np.int16)
    for trial in range(30):
        k = int(rng.integers(0, 12))
        st = np.sort(rng.uniform(0, 2000, k))
        segs = [(float(a), float(a + rng.uniform(-5, 300))) for a in st]
        rng.shuffle(segs)
        m_ref, out_ref = op.vad_merge(segs, samples)
        m_got, out_got = wdr.vad_merge(segs, samples)
        assert len(m_ref) == len(m_got)
        for (a, b), (c, d) in zip(m_ref, m_got):
            assert a == c and b == d
        assert len(out_ref) == len(out_got)
        for r, g in zip(out_ref, out_got):
            assert r.start == g.start and r.end == g.end
            np.testing.assert_array_equal(r.samples, g.samples)


def test_vad_merge_edge_cases():
    s = np.zeros(1000, np.int16)
    assert wdr.vad_merge([], s) == ([], [])
    m, out = wdr.vad_merge([(10.0, 5.0)], s)          # end <= start dropped
    assert m == [] and out == []
    m, out = wdr.vad_merge([(0.0, 100.0)], s)         # clamped to the sample count
    assert len(out) == 1 and out[0].samples.size == 1000


def test_synthetic_audio_is_deterministic():
    from wdr.synth import synth_speech
    a, sa = synth_speech(20.0, seed=1, n_speakers=3)
    b, sb = synth_speech(20.0, seed=1, n_speakers=3)
    np.testing.assert_array_equal(a, b)
    assert sa == sb and len(sa) >= 2
    assert {s[2] for s in sa} <= {0, 1, 2}
    for (s0, e0, _), (s1, e1, _) in zip(sa, sa[1:]):
        assert 1.5 - 1e-3 <= e0 - s0 <= 8.0 + 1e-3
        assert s1 - e0 >= 0.3 - 1e-3


def test_oracle_discrete_distribution_matches_libstdcxx(lib):
    """The t > 0 draw (whisper_sample_token: std::discrete_distribution + std::mt19937):
    oracle restatement vs the real libstdc++ through a host-only seam."""
    import ctypes as C
    from oracle.whisper_full import WhisperState
    rng = np.random.default_rng(3)
    for n, zeros in ((7, 0), (51866, 40000), (1, 0), (300, 299)):
        w = rng.random(n).astype(np.float32) ** 4
        if zeros:
            w[rng.choice(n, zeros, replace=False)] = 0
        if w.sum() == 0:
            w[-1] = 1
        out = np.zeros(64, np.int32)
        seed = int(rng.integers(0, 2 ** 31))
        _lib.check(lib.wdr_dbg_discrete(w.ctypes.data_as(C.POINTER(C.c_float)), n, seed, 64,
                                        out.ctypes.data_as(C.POINTER(C.c_int32))))
        rs = np.random.RandomState(seed)
        want = [WhisperState.discrete_draw(rs, w) for _ in range(64)]
        assert out.tolist() == want


def test_ggml_info_reads_whisper_cpp_header(tmp_path):
    """wdr_ggml_info parses a whisper.cpp ggml model file (the ggml-<model>.bin files
    src/model_manager.rs:162 caches and whisper-rs loads at src/transcribe.rs:154) without a GPU:
    header, mel filters, vocabulary and every tensor record."""
    from tests.ggml_writer import write_ggml
    p = str(tmp_path / "ggml-tiny-test.bin")
    hp, n_tensors, n_words, _ = write_ggml(p, "tiny-test")
    info = wdr.ggml_info(p)
    assert info["n_vocab"] == hp.n_vocab and info["n_mels"] == hp.n_mels
    assert (info["n_audio_state"], info["n_audio_layer"]) == (hp.n_audio_state, hp.n_audio_layer)
    assert (info["n_text_state"], info["n_text_layer"]) == (hp.n_text_state, hp.n_text_layer)
    assert info["ftype"] == 1
    assert info["n_tensors"] == n_tensors and info["n_vocab_tokens"] == n_words
    # f32 files parse too (ftype 0: every tensor f32)
    p32 = str(tmp_path / "ggml-f32.bin")
    write_ggml(p32, "tiny-test", ftype=0)
    assert wdr.ggml_info(p32)["ftype"] == 0


@pytest.mark.parametrize("kind,msg", [("magic", "bad magic"), ("trunc", "truncated"), ("missing", "doesn't exist")])
def test_ggml_info_rejects_bad_files(tmp_path, kind, msg):
    from tests.ggml_writer import write_ggml
    p = str(tmp_path / "m.bin")
    if kind == "magic":
        write_ggml(p, "tiny-test", magic=0x12345678)
    elif kind == "trunc":
        write_ggml(p, "tiny-test", truncate=5000)
    else:
        p = str(tmp_path / "absent.bin")
    with pytest.raises(wdr.WdrError, match=msg):
        wdr.ggml_info(p)


def test_shutdown_releases_handles_and_stale_calls_fail():
    """wdr_shutdown: a released handle is rejected by every entry point, freeing it is
    a no-op, and a handle created afterwards is a fresh one.  Run in a child process: shutdown
    releases every handle of the process."""
    import subprocess
    import sys
    code = r'''
import ctypes as C
from wdr import _lib as L
lib = L.load()
h = C.c_void_p()
assert lib.wdr_speakers_new(0, 0, C.byref(h)) == 0
emb = (C.c_float * 4)(1, 0, 0, 0)
buf = C.create_string_buffer(16)
assert lib.wdr_speakers_assign(h, emb, 4, 0.5, buf, 16) == 0 and buf.value == b"1"
lib.wdr_shutdown()
assert lib.wdr_speakers_assign(h, emb, 4, 0.5, buf, 16) != 0
assert b"released" in lib.wdr_last_error()
lib.wdr_speakers_free(h)          # no-op on a released handle
h2 = C.c_void_p()
assert lib.wdr_speakers_new(0, 0, C.byref(h2)) == 0 and h2.value != h.value
assert lib.wdr_speakers_assign(h2, emb, 4, 0.5, buf, 16) == 0 and buf.value == b"1"
lib.wdr_speakers_free(h2)
print("ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(root, "whisper-diarize-rs_amd"), root]))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout, r.stderr)


@pytest.mark.parametrize("v,n", [(None, 5), (0, 1), (-3, 1), (1, 1), (3, 3), (8, 8)])
def test_oracle_beam_size_default_matches_reference(v, n):
    """src/transcribe.rs:22: best_of_or_beam_size.unwrap_or(5).max(1) -- Some(0) is 1, not 5
    (libwdr csrc/engine.cpp setup_params reads it the same way)."""
    from oracle.pipeline import setup_params
    adv = {} if v is None else dict(best_of_or_beam_size=v)
    for strat in (None, "greedy"):
        if strat:
            adv = dict(adv, sampling_strategy=strat)
        p = setup_params(dict(advanced=adv))
        assert p.beam_size == p.best_of == n


def test_every_handle_entry_point_holds_its_handle():
    """every C entry point that takes an engine / vad / diarizer / speakers / context
    handle (other than *_free) takes a WDR_USE hold, so a released handle is rejected and an
    in-flight call is counted busy by wdr_shutdown (a source check: no GPU needed)."""
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "whisper-diarize-rs_amd", "csrc", "engine.cpp")).read()
    missing, n = [], 0
    for m in re.finditer(r"\n(?:int|void|size_t|double) (wdr_\w+)\(([^)]*)\)\s*\{", src):
        name, args = m.group(1), m.group(2)
        hs = re.findall(r"wdr_(engine|vad|diarizer|speakers|context)\*\s*(\w+)", args)
        if not hs or name.endswith("_free"):
            continue
        n += 1
        body = src[m.end():src.find("\n}\n", m.end())]
        if not all(re.search(r"WDR_USE\(\w+,\s*%s\)" % h, body) for _, h in hs):
            missing.append(name)
    assert n >= 25 and not missing, (n, missing)
