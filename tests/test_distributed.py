"""Multi-GPU one-file path (wdr/distributed.py) on CPU: world_size 2 over gloo.

The per-rank compute is the CPU oracle (test-only) on the tiny synthetic model, so the whole
exchange -- window shards of the segmentation, gather + stitching on rank 0, contiguous
segment blocks, the speculative decode + rank-ordered prompt fix-up, the gather and the
in-order merge (overlap clip, speakers, callbacks) -- is checked against ONE sequential run
of the same oracle over the whole file: segments must be identical (text, times, words,
speakers).  The GPU box runs the same code with the HIP pipeline (test_gpu_distributed.py)."""
import dataclasses
import json
import os
import socket

import numpy as np
import pytest

import wdr
from wdr import distributed as D

torch = pytest.importorskip("torch")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


OPTS = dict(lang="en", advanced=dict(sampling_strategy="greedy"),
            synthetic=dict(force_len_rate=3.3, logprob_thold=-np.inf, entropy_thold=-1.0))


def _oracle_state():
    from oracle.model import Whisper
    from oracle.vocab import Vocab
    from oracle.weights import hparams_for, synth_weights
    from oracle.whisper_full import WhisperState
    hp = hparams_for("tiny-test")
    return WhisperState(Whisper(hp, synth_weights(hp, std=0.02, emb_std=0.5)), Vocab(hp.n_vocab), "tiny-test")


def _to_wdr(segs):
    return [wdr.Segment(s.start, s.end, s.text,
                        [wdr.WordTimestamp(w.text, w.start, w.end, w.probability) for w in s.words] if s.words else None,
                        s.speaker_id) for s in segs]


def _oracle_block(state):
    from oracle.pipeline import SpeechSegment as OSeg
    from oracle.pipeline import run_transcription_pipeline

    def run(segs, prompt):
        opts = dict(OPTS, advanced=dict(OPTS["advanced"], init_prompt=prompt))
        groups, lang = run_transcription_pipeline(state, [OSeg(s.start, s.end, s.samples) for s in segs], opts, raw=True)
        return [_to_wdr(g) for g in groups], lang
    return run


def fake_classes(pcm):
    """Window-local stand-in for segmentation-3.0 (frame class from the frame's energy)."""
    n = pcm.size
    padded = np.zeros(n + (160000 - n % 160000), np.float32)
    padded[:n] = pcm
    W = padded.size // 160000
    out = np.zeros((W, 589), np.int32)
    for w in range(W):
        x = padded[w * 160000:(w + 1) * 160000]
        for k in range(589):
            f = x[k * 270:k * 270 + 721]
            out[w, k] = 1 if np.abs(f).mean() > 200 else 0
    return out


def fake_embed(samples):
    if samples.size < 400:
        return None
    rng = np.random.default_rng(int(np.abs(samples.astype(np.int64)).sum()) % (2 ** 32))
    return rng.standard_normal(512).astype(np.float32)


def _worker(rank, world, port, mode, pcm_path, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pcm = np.load(pcm_path) if rank == 0 else None
        opts = wdr.TranscribeOptions(lang="en", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
        got_cb = []
        cb = wdr.Callbacks(new_segment_callback=lambda s: got_cb.append(s.text))
        if mode == "vad":
            from wdr.synth import synth_speech  # noqa: F401
            spurts = json.load(open(pcm_path + ".json"))
            segf = lambda p: [wdr.SpeechSegment(a, b, p[int(round(a * 16000)):int(round(b * 16000))])
                              for a, b in spurts]
            res = D.transcribe_file(pcm, opts, segmentation="vad", block_fn=_oracle_block(_oracle_state()),
                                    speech_segments_fn=segf, callbacks=cb)
        else:
            res = D.transcribe_file(pcm, opts, segmentation="diarize", block_fn=_oracle_block(_oracle_state()),
                                    classes_fn=fake_classes, embed_fn=fake_embed, callbacks=cb)
        if rank == 0:
            segs, lang = res
            json.dump({"segs": [dataclasses.asdict(s) for s in segs], "lang": lang, "cb": got_cb},
                      open(out_path, "w"))
        else:
            assert res is None
    finally:
        torch.distributed.destroy_process_group()


def _sequential(pcm, mode, spurts):
    from oracle.pipeline import SpeechSegment as OSeg
    from oracle.pipeline import run_transcription_pipeline
    st = _oracle_state()
    if mode == "vad":
        segs = [OSeg(a, b, pcm[int(round(a * 16000)):int(round(b * 16000))]) for a, b in spurts]
    else:
        segs = [OSeg(s.start, s.end, s.samples) for s in wdr.Diarizer.segments_from_classes(fake_classes(pcm), pcm)]
    out, lang = run_transcription_pipeline(st, segs, OPTS)
    out = _to_wdr(out)
    if mode == "diarize":
        mgr = wdr.SpeakerManager(None)
        # every whisper segment of speech segment i gets embedding i, assigned in order
        from oracle.pipeline import run_transcription_pipeline as rtp
        groups, _ = rtp(_oracle_state(), segs, OPTS, raw=True)
        k = 0
        for i, g in enumerate(groups):
            e = fake_embed(segs[i].samples)
            for _ in g:
                out[k].speaker_id = mgr.assign(e, 0.5)
                k += 1
    return out, lang


@pytest.mark.parametrize("mode", ["vad", "diarize"])
def test_two_ranks_match_sequential(tmp_path, mode):
    from wdr.synth import synth_speech
    pcm, spurts = synth_speech(34.0, seed=5, n_speakers=2)
    spurts = [(a, b) for a, b, _ in spurts]
    p = str(tmp_path / "pcm.npy")
    np.save(p, pcm)
    json.dump(spurts, open(p + ".json", "w"))
    out = str(tmp_path / "out.json")
    torch.multiprocessing.spawn(_worker, args=(2, _port(), mode, p, out), nprocs=2, join=True)
    got = json.load(open(out))
    ref, lang = _sequential(pcm, mode, spurts)
    assert len(ref) >= 3
    assert got["lang"] == lang
    assert [s["text"] for s in got["segs"]] == [s.text for s in ref]
    for g, r in zip(got["segs"], ref):
        assert (g["start"], g["end"]) == (r.start, r.end)
        assert g["speaker_id"] == r.speaker_id
        gw = [(w["text"], w["start"], w["end"]) for w in (g["words"] or [])]
        rw = [(w.text, w.start, w.end) for w in (r.words or [])]
        assert gw == rw
    assert got["cb"] == [s.text for s in ref]


def _fake_block(segs, prompt):
    """Text depends on the prompt only for every third segment (id from the samples)."""
    groups = []
    e = prompt
    for s in segs:
        sid = int(s.samples[0])
        text = ("p%s|%d" % ((e or "-")[:3], sid)) if sid % 3 == 0 else ("" if sid % 5 == 0 else "s%d" % sid)
        g = [wdr.Segment(s.start, s.end, text)]
        groups.append(g)
        e = D.next_prompt(e, g)
    return groups, "en"


def _chain_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        segs = [wdr.SpeechSegment(float(i), i + 0.5, np.full(10, i, np.int16)) for i in range(40)]
        a, b = D.balance([1] * 40, world)[rank]
        calls = []

        def counted(ss, p):
            calls.append(len(ss))
            return _fake_block(ss, p)
        groups, _ = D.transcribe_block(counted, segs[a:b], None, rank, world, seg0=a)
        gathered = [None] * world if rank == 0 else None
        torch.distributed.gather_object(([g[0].text for g in groups], calls), gathered, dst=0)
        if rank == 0:
            json.dump(gathered, open(out_path, "w"))
    finally:
        torch.distributed.destroy_process_group()


def test_prompt_fixup_stops_at_convergence(tmp_path):
    out = str(tmp_path / "chain.json")
    torch.multiprocessing.spawn(_chain_worker, args=(4, _port(), out), nprocs=4, join=True)
    got = json.load(open(out))
    texts = sum([g[0] for g in got], [])
    segs = [wdr.SpeechSegment(float(i), i + 0.5, np.full(10, i, np.int16)) for i in range(40)]
    ref, _ = _fake_block(segs, None)
    assert texts == [g[0].text for g in ref]
    # ranks 1..3 re-decode only until the prompt converges (a few single-segment calls)
    for calls in [g[1] for g in got][1:]:
        assert calls[0] == 10 and all(c == 1 for c in calls[1:]) and len(calls) - 1 <= 4, calls


def _fake_block_rng(segs, prompt, rng):
    """Like _fake_block, and every 7th segment "draws": its text depends on the RNG counter (a
    string, as the mt19937 state is), which each draw advances.  rng None = the fresh state."""
    groups, sampled = [], []
    e = prompt
    r = int(rng) if rng is not None else 0
    for s in segs:
        sid = int(s.samples[0])
        if sid % 7 == 3:
            r += 1 + len(e or "") % 3
            text = "r%d|%d" % (r, sid)
            sampled.append(True)
        else:
            text = ("p%s|%d" % ((e or "-")[:3], sid)) if sid % 3 == 0 else ("" if sid % 5 == 0 else "s%d" % sid)
            sampled.append(False)
        g = [wdr.Segment(s.start, s.end, text)]
        groups.append(g)
        e = D.next_prompt(e, g)
    return groups, "en", sampled, str(r)


def _rng_worker(rank, world, port, out_path, n):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        segs = [wdr.SpeechSegment(float(i), i + 0.5, np.full(10, i, np.int16)) for i in range(n)]
        a, b = D.balance([1] * n, world)[rank]
        groups, _ = D.transcribe_block(_fake_block_rng, segs[a:b], None, rank, world, seg0=a)
        gathered = [None] * world if rank == 0 else None
        torch.distributed.gather_object(([g[0].text for g in groups], dict(D.last_stats)), gathered, dst=0)
        if rank == 0:
            json.dump(gathered, open(out_path, "w"))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,n", [(3, 40), (4, 9), (4, 3)])
def test_rng_replay_across_ranks(tmp_path, world, n):
    """Sampled segments (temperature fallback) make every later result depend on decoder 0's
    RNG stream: the multi-rank decode (parallel prompt rounds, then the in-order replay from the
    first segment that drew, RNG state handed rank to rank) equals one sequential pass; also
    with ranks that hold no segments (n < world)."""
    out = str(tmp_path / "rng.json")
    torch.multiprocessing.spawn(_rng_worker, args=(world, _port(), out, n), nprocs=world, join=True)
    got = json.load(open(out))
    texts = sum([g[0] for g in got], [])
    segs = [wdr.SpeechSegment(float(i), i + 0.5, np.full(10, i, np.int16)) for i in range(n)]
    ref = _fake_block_rng(segs, None, None)[0]
    assert texts == [g[0].text for g in ref]


def test_balance_partitions():
    r = D.balance([1] * 10, 4)
    assert r[0][0] == 0 and r[-1][1] == 10 and all(x[1] == y[0] for x, y in zip(r, r[1:]))
    assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1
    assert D.balance([], 3) == [(0, 0)] * 3
    r = D.balance([5, 1, 1, 1, 1, 1], 2)
    assert r[0][0] == 0 and r[-1][1] == 6 and all(x[1] == y[0] for x, y in zip(r, r[1:]))
