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
