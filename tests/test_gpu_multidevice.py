"""In-process multi-GPU (gpu_device None: every visible GPU, src/engine.rs:14 / SURVEY §8(b)):
one model per GPU, the decode chains spread over them (chain k on GPU k % G) with the exact
prompt fix-up across GPUs.  On a one-GPU machine WDR_DEVICES="0,0" puts two models (two KV
pools, two step batchers) on GPU 0, which runs the same cross-model code.  The result must
equal the one-GPU, one-chain pipeline exactly."""
import dataclasses

import pytest

import wdr
from wdr.synth import synth_speech

pytestmark = pytest.mark.gpu


def _segs(pcm, spurts):
    return [wdr.SpeechSegment(a, b, pcm[int(round(a * 16000)):int(round(b * 16000))]) for a, b, _ in spurts]


def _run(ctx, segs, opts, chains):
    ctx.set_chains(chains)
    out, lang = ctx.run_pipeline(segs, opts)
    return [dataclasses.asdict(s) for s in out], lang


def test_default_device_is_every_visible_gpu():
    import torch
    ctx = wdr.WhisperContext("tiny-test", synthetic=wdr.Synthetic())
    assert ctx.devices == list(range(min(torch.cuda.device_count(), 8)))
    ctx.close()
    ctx = wdr.WhisperContext("tiny-test", gpu_device=0, synthetic=wdr.Synthetic())
    assert ctx.devices == [0]
    ctx.close()


@pytest.mark.parametrize("name,seconds,strategy,chains", [
    ("tiny-test", 80.0, "greedy", 3),
    ("tiny-test", 60.0, None, 2),
    ("large-v3", 60.0, "greedy", 4),
])
def test_two_models_equal_one(name, seconds, strategy, chains, monkeypatch):
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)
    pcm, spurts = synth_speech(seconds, seed=9, n_speakers=2)
    segs = _segs(pcm, spurts)
    opts = wdr.TranscribeOptions(lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy=strategy))
    one = wdr.WhisperContext(name, gpu_device=0, synthetic=syn)
    ref, lang1 = _run(one, segs, opts, 1)
    one.close()
    monkeypatch.setenv("WDR_DEVICES", "0,0")
    two = wdr.WhisperContext(name, synthetic=syn)
    assert two.devices == [0, 0]
    got, lang = _run(two, segs, opts, chains)
    st = two.stage_times()
    assert st["chains"] == min(2 * chains, len(segs))
    assert lang == lang1
    assert got == ref
    two.close()


def _progress(**kw):
    """A line under gpurun_out/ between the phases of a long test (the GPU box treats minutes of
    silence as a hang)."""
    import json
    import os
    p = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "multidevice_progress.jsonl")
    try:
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "a") as f:
            f.write(json.dumps(kw) + "\n")
    except OSError:
        pass


@pytest.mark.timeout(1500)
def test_configs3_split_eight_logical_devices(monkeypatch):
    """BASELINE configs[3]'s split at full size on one GPU: a 4-h, 3-speaker large-v3 + DTW +
    diarization run (speaker embeddings + assignment) through run_pipeline with
    WDR_DEVICES=0,0,0,0,0,0,0,0 -- eight models, eight step batchers and DTW queues, 3 decode
    chains each: 24 speculative blocks over 8 "GPUs" and the exact prompt fix-up rounds across
    them (src/engine.rs:14, src/transcribe.rs:110-112) -- must equal one model with 24 chains bit
    for bit (which the chain tests pin to one chain).  Greedy decode (the bench's), so the 4 h
    fit the test's time."""
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.02, force_len_rate=3.3, disable_fallback=True)
    pcm, spurts = synth_speech(14400.0, seed=1, n_speakers=3)
    segs = _segs(pcm, spurts)
    _progress(phase="audio", segments=len(segs))
    opts = wdr.TranscribeOptions(model="large-v3", lang="auto", enable_vad=False, enable_diarize=True,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    dopts = wdr.DiarizeOptions.from_options(opts)
    one = wdr.WhisperContext("large-v3", gpu_device=0, enable_dtw=True, synthetic=syn)
    one.set_chains(24)
    ref, lang1 = one.run_pipeline(segs, opts, diarize_options=dopts)
    one.close()
    _progress(phase="one device", segments=len(ref))
    monkeypatch.setenv("WDR_DEVICES", ",".join(["0"] * 8))
    # the per-model pools (KV sequences, cross-K/V slot rings of the chains' states) are sized at
    # creation for WDR_DECODE_CHAINS chains: 3 per model here, or eight 24-chain pools would not
    # fit one GPU's 288 GB
    monkeypatch.setenv("WDR_DECODE_CHAINS", "3")
    eight = wdr.WhisperContext("large-v3", enable_dtw=True, synthetic=syn)
    assert eight.devices == [0] * 8
    eight.set_chains(3)
    got, lang = eight.run_pipeline(segs, opts, diarize_options=dopts)
    st = eight.stage_times()
    eight.close()
    _progress(phase="eight devices", segments=len(got), fixups=st.get("fixup_segments"), chains=st.get("chains"))
    assert st["chains"] == 24
    assert lang == lang1 and len(got) == len(ref) >= 2000
    assert [dataclasses.asdict(s) for s in got] == [dataclasses.asdict(s) for s in ref]


@pytest.mark.timeout(1500)
def test_configs4_eight_logical_devices_fp8(monkeypatch):
    """BASELINE configs[4] at full size on one GPU: 8 h of 4-speaker audio (seed 2,
    4 speakers), large-v3, lang auto, DTW, diarization (speaker embeddings + assignment), the fp8
    MX encoder GEMMs (k_gemm8), through WDR_DEVICES=0 x 8 -- eight models, 3 decode chains each,
    the exact prompt fix-up across them -- against one fp8 model with 24 chains: bit-identical
    output, and every segment holds the properties the reference's glue guarantees
    (tests/pipeline_props.py).  Greedy decode, as the bench."""
    from tests.pipeline_props import check_pipeline_properties
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.02, force_len_rate=3.3, disable_fallback=True)
    pcm, spurts = synth_speech(28800.0, seed=2, n_speakers=4)
    segs = _segs(pcm, spurts)
    _progress(phase="c4 audio", segments=len(segs))
    # speaker assignment with 4 speakers and the threshold that separates the synthetic voices
    # (make_pipeline_fixtures.py DIAR: at the default 0.5 every segment is speaker "1")
    opts = wdr.TranscribeOptions(model="large-v3", lang="auto", enable_vad=False, enable_diarize=True,
                                 max_speakers=4,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy", diarize_threshold=0.9999))
    dopts = wdr.DiarizeOptions.from_options(opts)
    one = wdr.WhisperContext("large-v3", gpu_device=0, enable_dtw=True, synthetic=syn)
    one.set_encoder_fp8(True)
    one.set_chains(24)
    ref, lang1 = one.run_pipeline(segs, opts, diarize_options=dopts)
    one.close()
    _progress(phase="c4 one device", segments=len(ref))
    speakers, words, inverted = check_pipeline_properties(ref, spurts)
    monkeypatch.setenv("WDR_DEVICES", ",".join(["0"] * 8))
    monkeypatch.setenv("WDR_DECODE_CHAINS", "3")
    eight = wdr.WhisperContext("large-v3", enable_dtw=True, synthetic=syn)
    assert eight.devices == [0] * 8
    eight.set_encoder_fp8(True)
    eight.set_chains(3)
    got, lang = eight.run_pipeline(segs, opts, diarize_options=dopts)
    st = eight.stage_times()
    eight.close()
    _progress(phase="c4 eight devices", segments=len(got), fixups=st.get("fixup_segments"), chains=st.get("chains"),
              speakers=speakers, words=words, inverted_words=inverted)
    assert st["chains"] == 24
    assert lang == lang1 and len(got) == len(ref) >= 4000
    assert [dataclasses.asdict(s) for s in got] == [dataclasses.asdict(s) for s in ref]
