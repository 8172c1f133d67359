"""One audio file across G GPUs: one process per GPU over torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for the CPU tests).

The reference transcribes a file on one device (src/engine.rs:65-200).  Here:

1. Rank 0 holds the file's PCM (`read_wav`).  Its length is broadcast.
2. Segmentation.  pyannote (src/engine.rs:89-122): its 10-s windows are independent, so the
   windows are split into G contiguous shards, each rank's PCM slice is scattered to it, every
   rank computes its windows' frame classes on its GPU, the classes are gathered to rank 0 and
   stitched there in file order (the stitching is sequential: frame offsets continue across
   windows).  Silero VAD carries its LSTM state across the whole file, so it runs on rank 0
   (0.2 s per hour of audio); no segmentation = one segment.
3. The speech segments are split into G contiguous blocks balanced by sample count; each
   rank receives its block's samples (scatter) and transcribes it on its GPU, while a host
   thread computes the block's speaker embeddings (diarize).
4. Prompt chain, exact.  Segment i's decode depends on the prompt E_i (src/transcribe.rs:384-386,
   502): E_{i+1} = the text of segment i's last result if that is non-empty, else E_i.  Every
   rank first decodes its block speculatively from the file's initial prompt.  Then fix-up
   rounds, all ranks at once: the prompts leaving every block are all-gathered; every rank whose
   block was decoded from a prompt other than the one leaving its predecessor's block (as that
   now stands) re-decodes its segments one at a time from it until the prompt entering the next
   segment equals the previous run's (from there on the previous results are the sequential
   ones).  A rank that ran through its block changes its successor's true prompt, which the next
   round handles; rank 0 is always exact, so the rounds end.  Random draws (t > 0 decoders:
   temperature fallback) make results depend on decoder 0's RNG stream, which in the reference
   runs through the whole file in one state: from the first segment that drew in any decode,
   the rest of the file is re-decoded in order, the RNG state and prompt handed from rank to
   rank (wdr_run_pipeline_block carries the state in and out).  The result equals the
   single-GPU run exactly.
5. Raw per-segment results (no overlap clip, no speakers: wdr_run_pipeline_raw) and
   embeddings are gathered to rank 0, which merges them in file order and applies what the
   reference does sequentially: the overlap clip of each segment against its successor
   (src/transcribe.rs:447-459), speaker assignment in order (src/transcribe.rs:461-497) and the
   callbacks (new_segment before the clip, then progress (i+1)/N*100).

The per-rank compute (`block_fn`, `classes_fn`, `embed_fn`) is injectable so the CPU tests run
the same exchange logic with world_size 2 on gloo.
"""
from __future__ import annotations

import dataclasses
import threading
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import Callbacks, ProgressType, Segment, SpeakerManager, SpeechSegment, TranscribeOptions, WordTimestamp

WIN = 160000          # pyannote window (10 s at 16 kHz)
FRAMES = 589          # segmentation-3.0 frames per window


# ------------------------------------------------------------------ collectives (device-aware)
def _dist():
    import torch.distributed as dist
    return dist


def _device():
    import torch
    dist = _dist()
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _t(a: np.ndarray):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(_device())


def _np(t) -> np.ndarray:
    return t.cpu().numpy()


def _bcast_i64(vals: Optional[Sequence[int]], n: int, src: int = 0) -> np.ndarray:
    import torch
    dist = _dist()
    t = _t(np.asarray(vals, np.int64)) if dist.get_rank() == src else torch.zeros(n, dtype=torch.int64,
                                                                                   device=_device())
    dist.broadcast(t, src)
    return _np(t)


def _bcast_array(a: Optional[np.ndarray], dtype, src: int = 0) -> np.ndarray:
    """Broadcast a 1-D or 2-D array of dtype from src (shape first)."""
    import torch
    dist = _dist()
    if dist.get_rank() == src:
        a = np.ascontiguousarray(a, dtype)
        shape = list(a.shape) + [1] * (2 - a.ndim)
    else:
        shape = [0, 0]
    shape = _bcast_i64(shape, 2, src)
    if dist.get_rank() == src:
        t = _t(a.reshape(shape))
    else:
        t = torch.zeros(tuple(int(x) for x in shape), dtype=getattr(torch, np.dtype(dtype).name), device=_device())
    dist.broadcast(t, src)
    return _np(t)


def _scatter_1d(parts: Optional[List[np.ndarray]], dtype, src: int = 0) -> np.ndarray:
    """Scatter G 1-D arrays of different lengths from src (moved as bytes, padded to the
    longest; gloo has no int16 collectives)."""
    import torch
    dist = _dist()
    G, rank = dist.get_world_size(), dist.get_rank()
    isz = np.dtype(dtype).itemsize
    raw = [np.ascontiguousarray(p, dtype).view(np.uint8) for p in parts] if rank == src else None
    lens = _bcast_i64([int(p.size) for p in raw] if rank == src else None, G, src)
    cap = max(isz, int(lens.max()))
    out = torch.zeros(cap, dtype=torch.uint8, device=_device())
    if rank == src:
        bufs = []
        for p in raw:
            b = np.zeros(cap, np.uint8)
            b[:p.size] = p
            bufs.append(_t(b))
        dist.scatter(out, bufs, src)
    else:
        dist.scatter(out, None, src)
    return _np(out)[:int(lens[rank])].copy().view(dtype)


def _gather_2d(a: np.ndarray, dtype, dst: int = 0) -> Optional[List[np.ndarray]]:
    """Gather 2-D arrays [n_r][C] of different row counts to dst (padded)."""
    import torch
    dist = _dist()
    G, rank = dist.get_world_size(), dist.get_rank()
    a = np.ascontiguousarray(a, dtype)
    C = a.shape[1]
    rows = torch.tensor([a.shape[0]], dtype=torch.int64, device=_device())
    all_rows = [torch.zeros(1, dtype=torch.int64, device=_device()) for _ in range(G)]
    dist.all_gather(all_rows, rows)
    cap = max(1, max(int(r.item()) for r in all_rows))
    buf = np.zeros((cap, C), dtype)
    buf[:a.shape[0]] = a
    tdt = getattr(torch, np.dtype(dtype).name)
    if rank == dst:
        outs = [torch.zeros((cap, C), dtype=tdt, device=_device()) for _ in range(G)]
        dist.gather(_t(buf), outs, dst)
        return [_np(o)[:int(r.item())] for o, r in zip(outs, all_rows)]
    dist.gather(_t(buf), None, dst)
    return None


def _send_prompt(p: Optional[str], dst: int):
    import torch
    dist = _dist()
    b = np.frombuffer(p.encode("utf-8"), np.uint8) if p is not None else np.zeros(0, np.uint8)
    n = torch.tensor([len(b) if p is not None else -1], dtype=torch.int64, device=_device())
    dist.send(n, dst)
    if b.size:
        dist.send(_t(b.copy()), dst)


def _recv_prompt(src: int) -> Optional[str]:
    import torch
    dist = _dist()
    n = torch.zeros(1, dtype=torch.int64, device=_device())
    dist.recv(n, src)
    k = int(n.item())
    if k < 0:
        return None
    if k == 0:
        return ""
    b = torch.zeros(k, dtype=torch.uint8, device=_device())
    dist.recv(b, src)
    return bytes(_np(b)).decode("utf-8")


# ------------------------------------------------------------------ partitioning / prompt chain
def balance(weights: Sequence[int], G: int) -> List[tuple]:
    """G contiguous index ranges [a, b) over len(weights) items with nearly equal weight sums
    (cut points at the k*total/G prefix quantiles); empty ranges allowed."""
    w = np.asarray(weights, np.float64)
    n = w.size
    if n == 0:
        return [(0, 0)] * G
    cum = np.concatenate([[0.0], np.cumsum(w)])
    cuts = [0]
    for k in range(1, G):
        t = cum[-1] * k / G
        c = int(np.searchsorted(cum, t, side="left"))
        if c > 0 and t - cum[c - 1] <= cum[min(c, n)] - t:   # nearest prefix sum, ties to the lower cut
            c -= 1
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[i], cuts[i + 1]) for i in range(G)]


def next_prompt(e_in: Optional[str], results: Sequence[Segment]) -> Optional[str]:
    """Prompt entering the next segment (src/transcribe.rs:384-386, 502): the text of this
    segment's last result when non-empty, else unchanged."""
    if results and results[-1].text.strip():
        return results[-1].text
    return e_in


def _raw_block(ctx, options: TranscribeOptions):
    """Default block transcriber: wdr_run_pipeline_block on this rank's GPU (decode chains,
    decoder 0's RNG carried in and out), results grouped per speech segment."""
    def run(segs: List[SpeechSegment], prompt: Optional[str], rng: Optional[str] = None) -> tuple:
        adv = dataclasses.replace(options.advanced) if options.advanced else None
        if adv is None:
            from . import AdvancedTranscribe
            adv = AdvancedTranscribe()
        adv.init_prompt = prompt
        opts = dataclasses.replace(options, advanced=adv, enable_diarize=None)
        out, lang, index, sampled, rng_out = ctx.run_pipeline_block(segs, opts, rng)
        groups: List[List[Segment]] = [[] for _ in segs]
        for s, i in zip(out, index):
            groups[i].append(s)
        return groups, lang, sampled, rng_out
    return run


def _as_block(fn):
    """block_fn(segs, prompt, rng) -> (groups, lang, sampled flags, rng after); a 2-argument
    function returning (groups, lang) is taken as one that never draws random numbers.  The
    arity is decided once from the signature: an error raised inside the block is never retried
    (a retry without the RNG state would silently change sampled results)."""
    import inspect
    try:
        params = inspect.signature(fn).parameters.values()
        positional = [p for p in params if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
        takes_rng = len(positional) >= 3 or any(p.kind == p.VAR_POSITIONAL for p in params)
    except (TypeError, ValueError):   # builtins without a signature: the documented 3-argument form
        takes_rng = True

    def run(segs, prompt, rng):
        r = fn(segs, prompt, rng) if takes_rng else fn(segs, prompt)
        if len(r) == 2:
            return r[0], r[1], [False] * len(segs), rng
        return r
    return run


# per-call statistics of the last transcribe_block on this rank (bench / probes)
last_stats: dict = {}


def _prompts(e0, groups):
    """Prompt entering each segment (and leaving the last): len(groups) + 1 entries."""
    out = [e0]
    for g in groups:
        out.append(next_prompt(out[-1], g))
    return out


def transcribe_block(block_fn, segs: List[SpeechSegment], spec_prompt: Optional[str], rank: int, G: int,
                     seg0: int = 0):
    """Speculative decode of this rank's block (its first segment is segment seg0 of the file),
    the parallel prompt fix-up rounds, then the in-order re-decode from the first segment that
    drew random numbers.  Returns (groups per speech segment, detected_lang of the block's first
    segment)."""
    import time
    dist = _dist()
    block = _as_block(block_fn)
    t0 = time.perf_counter()
    groups, lang, sampled, _ = block(segs, spec_prompt, None) if segs else ([], None, [], None)
    drew = list(sampled)                      # drew in any decode of the segment
    t1 = time.perf_counter()
    last_stats.clear()
    last_stats.update(segments=len(segs), spec_s=t1 - t0, fixups=0, rounds=0, replayed=0)
    dec_in = spec_prompt                      # the prompt this block's first segment was decoded from
    while True:
        states = [None] * G
        dist.all_gather_object(states, (dec_in, _prompts(dec_in, groups)[-1]))
        e_true = spec_prompt if rank == 0 else states[rank - 1][1]
        # a rank with no segments passes its predecessor's prompt on unchanged
        redo = bool(segs) and e_true != dec_in
        if not segs:
            dec_in = e_true
        flags = [None] * G
        dist.all_gather_object(flags, (redo, not segs and e_true != states[rank][0]))
        if not any(f[0] or f[1] for f in flags):
            break
        last_stats["rounds"] += 1
        if redo:
            spec_in = _prompts(dec_in, groups)
            e = e_true
            for j in range(len(segs)):
                last_stats["fixups"] += 1
                gj, lj, sj, _ = block([segs[j]], e, None)
                groups[j] = gj[0]
                drew[j] = drew[j] or sj[0]
                if j == 0:
                    lang = lj
                e = next_prompt(e, gj[0])
                if e == spec_in[j + 1]:
                    break
            dec_in = e_true
    t2 = time.perf_counter()
    last_stats.update(fixup_s=t2 - t1)
    # random draws: the first segment (file order) that drew in any decode is exact (nothing
    # before it drew, so it started from the fresh RNG); everything after it is re-decoded in
    # order with the RNG stream, block by block
    every = [None] * G
    dist.all_gather_object(every, (seg0, drew))
    first = None
    for s0, d in sorted(every, key=lambda x: x[0]):
        for k, x in enumerate(d):
            if x:
                first = s0 + k
                break
        if first is not None:
            break
    if first is not None:
        owner = next(r for r in range(G) if every[r][0] <= first < every[r][0] + len(every[r][1]))
        if rank == owner:
            k = first - seg0
            e = _prompts(dec_in, groups)[k]
            gk, lk, _, rng = block(segs[k:], e, None)
            groups[k:] = gk
            if k == 0:
                lang = lk
            last_stats["replayed"] += len(segs) - k
        elif rank > owner and segs:
            e = _recv_prompt(rank - 1)
            rng = _recv_prompt(rank - 1)
            groups, lang, _, rng = block(segs, e, rng)
            last_stats["replayed"] += len(segs)
        elif rank > owner:
            e = _recv_prompt(rank - 1)
            rng = _recv_prompt(rank - 1)
        if rank >= owner and rank < G - 1:
            e_out = _prompts(e, groups[k:] if rank == owner else groups)[-1]
            _send_prompt(e_out, rank + 1)
            _send_prompt(rng, rank + 1)
    last_stats.update(replay_s=time.perf_counter() - t2)
    return groups, lang


def merge_results(groups: List[List[Segment]], embeddings: Optional[List[Optional[np.ndarray]]],
                  threshold: float, max_speakers: Optional[int], n_speech: int,
                  callbacks: Optional[Callbacks] = None) -> List[Segment]:
    """Rank 0: the reference's sequential finishing over raw per-speech-segment results in file
    order: speaker per whisper segment (src/transcribe.rs:461-497), new_segment callback,
    overlap clip of the previous segment (src/transcribe.rs:447-459), progress (:518-522)."""
    mgr = SpeakerManager(max_speakers) if embeddings is not None else None
    out: List[Segment] = []
    for i, g in enumerate(groups):
        for s in g:
            s = dataclasses.replace(s, words=[dataclasses.replace(w) for w in s.words] if s.words else s.words)
            if out:
                last = out[-1]
                if last.end > s.start:
                    last.end = s.start
                if last.words and last.words[-1].end > last.end:
                    last.words[-1].end = last.end
            if mgr is not None:
                s.speaker_id = mgr.assign(embeddings[i], threshold)
            if callbacks and callbacks.new_segment_callback:
                callbacks.new_segment_callback(dataclasses.replace(s))
            if callbacks and callbacks.progress:
                callbacks.progress(int((i + 1) / max(1, n_speech) * 100), ProgressType.Transcribe,
                                   "Transcribing audio")
            out.append(s)
    return out


# ------------------------------------------------------------------ the whole call
def transcribe_file(pcm: Optional[np.ndarray], options: TranscribeOptions, *, ctx=None,
                    segmentation: str = "diarize", diarizer=None, vad=None,
                    callbacks: Optional[Callbacks] = None,
                    block_fn: Optional[Callable] = None, classes_fn: Optional[Callable] = None,
                    embed_fn: Optional[Callable] = None, speech_segments_fn: Optional[Callable] = None):
    """Transcribe ONE file on every rank of the default process group.  Rank 0 passes the
    file's int16 PCM, the other ranks None.  Returns (segments, detected_lang) on rank 0 and
    None elsewhere.  segmentation: "diarize" (pyannote, sharded by window), "vad" (Silero on
    rank 0) or "none" (whole file).  Speakers are assigned when segmentation == "diarize"."""
    dist = _dist()
    rank, G = dist.get_rank(), dist.get_world_size()
    if block_fn is None:
        block_fn = _raw_block(ctx, options)
    if classes_fn is None and segmentation == "diarize":
        classes_fn = diarizer.frame_classes
    n = int(_bcast_i64([int(pcm.size)] if rank == 0 else None, 1)[0])

    # ---- segmentation -> speech segments on rank 0
    segs: Optional[List[SpeechSegment]] = None
    if segmentation == "diarize":
        W = n // WIN + 1
        wr = balance([1] * W, G)
        parts = [pcm[a * WIN:min(n, b * WIN)] for a, b in wr] if rank == 0 else None
        mine = _scatter_1d(parts, np.int16)
        a, b = wr[rank]
        if b > a:
            cls = np.asarray(classes_fn(mine), np.int32).reshape(-1, FRAMES)[:b - a]
        else:
            cls = np.zeros((0, FRAMES), np.int32)
        allc = _gather_2d(cls, np.int32)
        if rank == 0:
            from . import Diarizer
            stitch = speech_segments_fn or Diarizer.segments_from_classes
            segs = stitch(np.concatenate(allc, 0), pcm)
    elif rank == 0:
        if segmentation == "vad":
            segs = speech_segments_fn(pcm) if speech_segments_fn else vad.get_segments(pcm)[1]
        else:
            segs = [SpeechSegment(0.0, n / 16000.0, pcm)]

    # ---- segment table + contiguous blocks
    if rank == 0:
        table = np.array([[s.start, s.end, s.samples.size] for s in segs], np.float64).reshape(-1, 3)
    table = _bcast_array(table if rank == 0 else None, np.float64)
    table = table.reshape(-1, 3) if table.size else np.zeros((0, 3))
    n_speech = table.shape[0]
    blocks = balance([int(x) for x in table[:, 2]], G)
    a, b = blocks[rank]
    parts = [np.concatenate([segs[i].samples for i in range(x, y)]).astype(np.int16) if y > x else
             np.zeros(0, np.int16) for x, y in blocks] if rank == 0 else None
    mine = _scatter_1d(parts, np.int16)
    my_segs, off = [], 0
    for i in range(a, b):
        k = int(table[i, 2])
        my_segs.append(SpeechSegment(float(table[i, 0]), float(table[i, 1]), mine[off:off + k]))
        off += k

    # ---- speaker embeddings beside the decode (host thread; the GPU call releases the GIL)
    embs: List[Optional[np.ndarray]] = [None] * len(my_segs)
    th = None
    if segmentation == "diarize":
        def work():
            batch = diarizer.embedding_batch if embed_fn is None else None
            if batch is not None:   # one batched CAM++ forward per 64 utterances
                for j in range(0, len(my_segs), 64):
                    embs[j:j + 64] = batch([s.samples for s in my_segs[j:j + 64]])
                return
            for j, s in enumerate(my_segs):
                embs[j] = embed_fn(s.samples)
        th = threading.Thread(target=work)
        th.start()
    spec = options.advanced.init_prompt if options.advanced else None
    try:
        groups, lang = transcribe_block(block_fn, my_segs, spec, rank, G, seg0=a)
    finally:
        if th is not None:
            th.join()

    # ---- gather to rank 0
    payload = (a, groups, lang)
    gathered = [None] * G if rank == 0 else None
    dist.gather_object(payload, gathered, dst=0)
    emb_all = None
    if segmentation == "diarize":
        E = np.zeros((len(my_segs), 513), np.float32)
        for j, e in enumerate(embs):
            if e is not None:
                E[j, :512] = e
                E[j, 512] = 1.0
        got = _gather_2d(E, np.float32)
        if rank == 0:
            allE = np.concatenate(got, 0)
            emb_all = [allE[i, :512].copy() if allE[i, 512] > 0 else None for i in range(n_speech)]
    if rank != 0:
        return None
    all_groups: List[List[Segment]] = []
    detected = None
    for a_r, g_r, l_r in sorted(gathered, key=lambda x: x[0]):
        if a_r == 0 and g_r:
            detected = l_r
        all_groups.extend(g_r)
    if options.lang and options.lang != "auto":
        detected = options.lang
    adv = options.advanced
    thr = adv.diarize_threshold if adv and adv.diarize_threshold is not None else 0.5
    max_spk = options.max_speakers if options.max_speakers else None
    out = merge_results(all_groups, emb_all, thr, max_spk, n_speech, callbacks)
    return out, detected
