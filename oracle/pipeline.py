"""The reference crate's own Rust glue, restated exactly (oracle side).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* `read_wav`                     <- src/audio.rs:4-24
* `vad_merge`                    <- src/vad.rs:33-84 (after segments_from_samples)
* `is_whole_control_token`,
  `strip_embedded_control_markers`,
  `get_token_timestamps`,
  `interpolate_word_timestamps`  <- src/transcribe.rs:171-320
* `run_transcription_pipeline`   <- src/transcribe.rs:323-535
* `transcribe_audio`             <- src/engine.rs:65-200 (segmentation choice + pipeline;
                                    translation and subtitle formatting are out of scope)
"""
from __future__ import annotations

import dataclasses
import struct

import numpy as np

from .mel import pcm_i16_to_f32
from .whisper_full import FullParams, WhisperState


@dataclasses.dataclass
class SpeechSegment:
    start: float
    end: float
    samples: np.ndarray


@dataclasses.dataclass
class Word:
    text: str
    start: float
    end: float
    probability: float | None = None


@dataclasses.dataclass
class Segment:
    start: float
    end: float
    text: str
    words: list | None = None
    speaker_id: str | None = None


class WavError(Exception):
    pass


def read_wav(path: str) -> np.ndarray:
    """hound WavReader + the reference's format checks (messages verbatim)."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise WavError("failed to read file")
    pos = 12
    fmt = None
    pcm = None
    while pos + 8 <= len(data):
        cid = data[pos:pos + 4]
        size = struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise WavError("failed to read file")
    tag, channels, rate, _, _, bits = fmt
    if channels != 1:
        raise WavError("expected mono audio file and found %d channels!" % channels)
    if tag not in (1, 0xFFFE):
        raise WavError("expected integer sample format")
    if rate != 16000:
        raise WavError("expected 16KHz sample rate")
    if bits != 16:
        raise WavError("expected 16 bits per sample")
    return np.frombuffer(pcm[:len(pcm) // 2 * 2], dtype="<i2").astype(np.int16)


def write_wav(path: str, samples: np.ndarray):
    s = np.asarray(samples, np.int16).tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(s)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, 16000, 32000, 2, 16)
    hdr += b"data" + struct.pack("<I", len(s))
    with open(path, "wb") as f:
        f.write(hdr + s)


def vad_merge(segs_cs, int_samples: np.ndarray):
    """src/vad.rs:33-84.  segs_cs: list of (start_cs, end_cs) floats from segments_from_samples."""
    n = int_samples.shape[0]
    SR = np.float32(16000.0)
    n_f32 = np.float32(n)
    mask = [(float(np.float32(s)) / 100.0, float(np.float32(e)) / 100.0) for s, e in segs_cs]
    mask = [(a, b) for a, b in mask if b > a]
    mask.sort(key=lambda t: t[0])
    merged = []
    for st, en in mask:
        if merged and st - merged[-1][1] < 0.200:
            merged[-1] = (merged[-1][0], max(en, merged[-1][1]))
        else:
            merged.append((st, en))
    out = []
    def rround(v):   # Rust f32::round: half away from zero
        v = float(v)
        return float(np.sign(v) * np.floor(abs(v) + 0.5))
    for st, en in merged:
        si = int(min(max(rround(np.float32(st) * SR), 0.0), float(n_f32)))
        ei = int(min(max(rround(np.float32(en) * SR), 0.0), float(n_f32)))
        smp = int_samples[si:ei].copy() if ei > si else np.zeros(0, np.int16)
        seg = SpeechSegment(st, en, smp)
        if seg.end > seg.start and smp.size > 0:
            out.append(seg)
    return mask, out


def is_whole_control_token(s: str) -> bool:
    t = s.strip("\0").strip()
    if not (t.startswith("[_") and t.endswith("]")):
        return False
    inner = t[2:-1]
    return len(inner) > 0 and all(c.isascii() and (c.isupper() or c.isdigit() or c == "_") for c in inner)


def strip_embedded_control_markers(s: str) -> str:
    out = []
    i, chars = 0, list(s)
    while i < len(chars):
        if i + 1 < len(chars) and chars[i] == "[" and chars[i + 1] == "_":
            j = i + 2
            while j < len(chars) and chars[j] != "]":
                j += 1
            if j < len(chars):
                if is_whole_control_token("".join(chars[i:j + 1])):
                    i = j + 1
                    continue
        out.append(chars[i])
        i += 1
    return "".join(out)


def cs_to_s(cs: int) -> float:
    return cs * 0.01


def get_token_timestamps(tokens, vocab):
    toks = []
    for t in tokens:
        raw = vocab.id_to_token[t.id]
        if is_whole_control_token(raw):
            continue
        clean = strip_embedded_control_markers(raw)
        if clean.strip("\0").strip() == "":
            continue
        anchor = cs_to_s(t.t_dtw) if t.t_dtw >= 0 else None
        toks.append((clean, float(np.float32(t.p)), cs_to_s(t.t0), cs_to_s(t.t1), anchor))
    if not toks:
        return []
    out = []
    for i, (text, p, t0, t1, a) in enumerate(toks):
        a_prev = toks[i - 1][4] if i > 0 else None
        a_next = toks[i + 1][4] if i + 1 < len(toks) else None
        start = 0.5 * (a_prev + a) if (a_prev is not None and a is not None) else t0
        end = 0.5 * (a + a_next) if (a is not None and a_next is not None) else t1
        out.append(Word(text, start, end, p))
    return out


def interpolate_word_timestamps(line: str, start: float, end: float):
    dur = max(end - start, 0.0)
    if dur <= 0.0:
        return []
    toks = [t for t in line.split() if t.strip("\0").strip()]
    if not toks:
        return []
    weights = [max(1, sum(1 for c in t if c.isalnum())) for t in toks]
    tot = sum(weights)
    out, acc = [], 0
    for i, t in enumerate(toks):
        a = start + (acc / tot) * dur
        b = end if i + 1 == len(toks) else start + ((acc + weights[i]) / tot) * dur
        acc += weights[i]
        out.append(Word(t, a, b, None))
    return out


def setup_params(options: dict) -> FullParams:
    """src/transcribe.rs:20-87 (the subset the options drive)."""
    adv = options.get("advanced") or {}
    v = adv.get("best_of_or_beam_size")
    n = max(1, 5 if v is None else v)   # unwrap_or(5).max(1): Some(0) -> 1, None -> 5
    p = FullParams()
    p.strategy = "greedy" if adv.get("sampling_strategy") == "greedy" else "beam"
    p.best_of = n
    p.beam_size = n
    if options.get("lang") is not None:
        p.language = options["lang"]
    if options.get("whisper_to_english"):
        p.translate = True
    if adv.get("temperature") is not None:
        p.temperature = adv["temperature"]
    if adv.get("max_text_ctx") is not None:
        p.n_max_text_ctx = adv["max_text_ctx"]
    if adv.get("init_prompt") is not None:
        p.initial_prompt = adv["init_prompt"]
    syn = options.get("synthetic") or {}
    for k, v in syn.items():
        setattr(p, k, v)
    return p


def run_transcription_pipeline(state: WhisperState, speech_segments, options: dict, raw: bool = False,
                               speaker_of=None):
    """src/transcribe.rs:323-535.  Returns (segments, detected_lang).
    raw: no overlap clip against the next segment; returns (results grouped per speech
    segment, detected_lang) -- the form wdr_run_pipeline_raw / the multi-GPU merge use.
    speaker_of(i): diarization (src/transcribe.rs:461-497) -- called once per whisper segment of
    speech segment i, in order (the reference recomputes the embedding of the speech segment's
    samples for every whisper segment and assigns it through the EmbeddingManager)."""
    vocab = state.v
    params = setup_params(options)
    user_offset = options.get("offset") or 0.0
    segments = []
    previous_text = None
    detected_lang = None
    lang = options.get("lang")
    if lang is not None and lang != "auto":
        detected_lang = lang
    translated = bool(options.get("whisper_to_english"))
    groups = []
    for i, ss in enumerate(speech_segments):
        groups.append([])
        samples = pcm_i16_to_f32(ss.samples)
        if previous_text is not None:
            params.initial_prompt = previous_text
        state.full(samples, params)
        if detected_lang is None:
            from .vocab import LANGS
            detected_lang = LANGS[state.lang_id]
        base_offset = ss.start + user_offset
        for res in state.result_all:
            text = res.text.lstrip()
            approx_start = base_offset + cs_to_s(res.t0)
            approx_end = base_offset + cs_to_s(res.t1)
            if translated:
                words = interpolate_word_timestamps(text, approx_start, approx_end)
            else:
                words = get_token_timestamps(res.tokens, vocab)
                for w in words:
                    w.start += base_offset
                    w.end += base_offset
            seg_start = words[0].start if words else approx_start
            seg_end = words[-1].end if words else approx_end
            if segments and not raw:
                last = segments[-1]
                if last.end > seg_start:
                    last.end = seg_start
                if last.words:
                    if last.words[-1].end > last.end:
                        last.words[-1].end = last.end
            previous_text = text if text.strip() else None
            spk = speaker_of(i) if speaker_of is not None else None
            segments.append(Segment(seg_start, seg_end, text, words or None, spk))
            groups[-1].append(segments[-1])
    if raw:
        return groups, detected_lang
    return segments, detected_lang
