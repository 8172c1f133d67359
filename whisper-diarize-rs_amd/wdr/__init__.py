"""Python mirror of the whisper-diarize-rs public API over libwdr's C ABI.

Same names, argument meaning and error behaviour as the reference crate
(src/lib.rs:12-17 re-exports; src/types.rs; src/engine.rs), so a caller of
`Engine::transcribe_audio` finds the same surface.  Every call goes through
libwdr.so (HIP, gfx950); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import enum
from typing import Callable, List, Optional

import numpy as np

from . import _lib as L

__all__ = ["Engine", "EngineConfig", "TranscribeOptions", "AdvancedTranscribe", "DiarizeOptions", "Segment",
           "WordTimestamp",
           "ProgressType", "Callbacks", "Synthetic", "WhisperContext", "SpeechSegment", "read_wav", "vad_merge",
           "WdrError"]

WdrError = L.WdrError


class ProgressType(enum.IntEnum):          # src/types.rs:5-9
    Download = 0
    Transcribe = 1
    Translate = 2


@dataclasses.dataclass
class AdvancedTranscribe:                  # src/types.rs:16-24
    sampling_strategy: Optional[str] = None
    best_of_or_beam_size: Optional[int] = None
    n_threads: Optional[int] = None
    temperature: Optional[float] = None
    max_text_ctx: Optional[int] = None
    init_prompt: Optional[str] = None
    diarize_threshold: Optional[float] = None


@dataclasses.dataclass
class TranscribeOptions:                   # src/types.rs:28-61 (defaults)
    offset: Optional[float] = 0.0
    model: str = "base"
    lang: Optional[str] = "auto"
    whisper_to_english: Optional[bool] = False
    translate_target: Optional[str] = None
    enable_vad: Optional[bool] = True
    enable_diarize: Optional[bool] = None
    max_speakers: Optional[int] = None
    advanced: Optional[AdvancedTranscribe] = None


@dataclasses.dataclass
class WordTimestamp:                       # src/types.rs:64-70
    text: str
    start: float
    end: float
    probability: Optional[float] = None


@dataclasses.dataclass
class Segment:                             # src/types.rs:74-82
    start: float
    end: float
    text: str
    words: Optional[List[WordTimestamp]] = None
    speaker_id: Optional[str] = None


@dataclasses.dataclass
class SpeechSegment:                       # src/types.rs:86-90
    start: float
    end: float
    samples: np.ndarray


@dataclasses.dataclass
class EngineConfig:                        # src/engine.rs:9-33 (defaults)
    cache_dir: str = "./cache"
    enable_dtw: Optional[bool] = True
    enable_flash_attn: Optional[bool] = False
    use_gpu: Optional[bool] = True
    gpu_device: Optional[int] = None
    vad_model_path: Optional[str] = None
    diarize_segment_model_path: Optional[str] = None
    diarize_embedding_model_path: Optional[str] = None


@dataclasses.dataclass
class Callbacks:                           # src/engine.rs:35-40
    progress: Optional[Callable[[int, ProgressType, str], None]] = None
    new_segment_callback: Optional[Callable[[Segment], None]] = None
    is_cancelled: Optional[Callable[[], bool]] = None


@dataclasses.dataclass
class DiarizeOptions:                      # src/types.rs:93-98
    """Passed to run_transcription_pipeline to switch speakers on (src/transcribe.rs:339-345).
    A None model path selects synthetic seeded weights (no model files offline)."""
    segment_model_path: Optional[str] = None
    embedding_model_path: Optional[str] = None
    threshold: float = 0.5
    max_speakers: int = 2 ** 64 - 1      # usize::MAX, the Engine's mapping of None / Some(0)

    @staticmethod
    def from_options(o: "TranscribeOptions", segment_model_path=None, embedding_model_path=None):
        """The DiarizeOptions Engine::transcribe_audio builds (src/engine.rs:101-111)."""
        thr = o.advanced.diarize_threshold if (o.advanced and o.advanced.diarize_threshold is not None) else 0.5
        mx = o.max_speakers if o.max_speakers else 2 ** 64 - 1
        return DiarizeOptions(segment_model_path, embedding_model_path, thr, mx)


def _dopts(d: Optional[DiarizeOptions], keep):
    if d is None:
        return None
    return keep(L.DiarizeOptions(keep(_s(d.segment_model_path)), keep(_s(d.embedding_model_path)), d.threshold,
                                 d.max_speakers))


@dataclasses.dataclass
class Synthetic:
    """Synthetic-weight / workload-pin knobs (no checkpoints here)."""
    weight_std: float = 0.02
    emb_std: float = 0.02
    force_len_rate: float = 0.0
    disable_fallback: bool = False


def _ob(v):
    return -1 if v is None else (1 if v else 0)


def _s(v):
    return None if v is None else v.encode()


class _Keep:
    """Keeps ctypes buffers alive for the duration of a call."""

    def __init__(self):
        self.objs = []

    def __call__(self, o):
        self.objs.append(o)
        return o


def _opts(o: Optional[TranscribeOptions], keep: _Keep):
    if o is None:
        return None
    t = L.TranscribeOptions()
    t.has_offset = 0 if o.offset is None else 1
    t.offset = o.offset or 0.0
    t.model = keep(_s(o.model))
    t.lang = keep(_s(o.lang))
    t.whisper_to_english = _ob(o.whisper_to_english)
    t.translate_target = keep(_s(o.translate_target))
    t.enable_vad = _ob(o.enable_vad)
    t.enable_diarize = _ob(o.enable_diarize)
    t.has_max_speakers = 0 if o.max_speakers is None else 1
    t.max_speakers = o.max_speakers or 0
    if o.advanced is not None:
        a = o.advanced
        A = L.Advanced()
        A.sampling_strategy = keep(_s(a.sampling_strategy))
        for f in ("best_of_or_beam_size", "n_threads", "temperature", "max_text_ctx", "diarize_threshold"):
            v = getattr(a, f)
            setattr(A, "has_" + f, 0 if v is None else 1)
            setattr(A, f, v or 0)
        A.init_prompt = keep(_s(a.init_prompt))
        keep(A)
        t.advanced = C.pointer(A)
    return keep(t)


def _syn(s: Optional[Synthetic]):
    if s is None:
        return None
    return L.Synthetic(s.weight_std, s.emb_std, s.force_len_rate, 1 if s.disable_fallback else 0)


@dataclasses.dataclass
class FormattingOverrides:                 # src/formatting.rs:37-51
    max_chars_per_line: Optional[int] = None
    max_lines: Optional[int] = None
    cps_cap: Optional[float] = None
    split_gap_sec: Optional[float] = None
    comma_min_chars_before_allow: Optional[int] = None
    min_word_dur: Optional[float] = None
    min_sub_dur: Optional[float] = None
    max_sub_dur: Optional[float] = None
    soft_max_words_per_line: Optional[int] = None
    insert_interword_space: Optional[bool] = None
    use_grapheme_len: Optional[bool] = None
    enforce_kinsoku: Optional[bool] = None
    allow_comma_split: Optional[bool] = None


def _fmt(ov: Optional[FormattingOverrides]):
    if ov is None:
        return None
    f = L.FormattingOverrides()
    for name in ("max_chars_per_line", "max_lines", "cps_cap", "split_gap_sec", "comma_min_chars_before_allow",
                 "min_word_dur", "min_sub_dur", "max_sub_dur", "soft_max_words_per_line"):
        v = getattr(ov, name)
        setattr(f, "has_" + name, 0 if v is None else 1)
        setattr(f, name, v or 0)
    for name in ("insert_interword_space", "use_grapheme_len", "enforce_kinsoku", "allow_comma_split"):
        setattr(f, name, _ob(getattr(ov, name)))
    return f


def _raw_segments(segs: List[Segment], keep: "_Keep"):
    arr = (L.Segment * max(1, len(segs)))()
    for i, sg in enumerate(segs):
        arr[i].start, arr[i].end = sg.start, sg.end
        arr[i].text = keep(sg.text.encode())
        if sg.words is not None:
            w = (L.Word * max(1, len(sg.words)))()
            for k, x in enumerate(sg.words):
                w[k].text = keep(x.text.encode())
                w[k].start, w[k].end = x.start, x.end
                w[k].has_probability = 0 if x.probability is None else 1
                w[k].probability = x.probability or 0.0
            keep(w)
            arr[i].words = C.cast(w, C.POINTER(L.Word))
            arr[i].n_words = len(sg.words)
        arr[i].speaker_id = keep(None if sg.speaker_id is None else sg.speaker_id.encode())
    keep(arr)
    return arr


def process_segments(segments: List[Segment], lang: str = "auto", overrides: Optional[FormattingOverrides] = None,
                     vad_mask=None) -> List[Segment]:
    """formatting::process_segments with PostProcessConfig::for_language(lang) + overrides and
    an optional VAD mask oracle (src/engine.rs:192-199)."""
    lib = L.load()
    keep = _Keep()
    arr = _raw_segments(segments, keep)
    ov = _fmt(overrides)
    m = np.ascontiguousarray(np.asarray(vad_mask if vad_mask is not None else [], np.float64).reshape(-1))
    out = C.POINTER(L.SegmentList)()
    L.check(lib.wdr_process_segments(arr, len(segments), lang.encode(), C.byref(ov) if ov is not None else None,
                                     0 if vad_mask is None else 1, m.ctypes.data_as(C.POINTER(C.c_double)),
                                     m.size // 2, C.byref(out)))
    return _segments(out)[0]


def _segments(lst_ptr, with_index: bool = False) -> tuple:
    lst = lst_ptr.contents
    index = [int(lst.speech_index[i]) for i in range(lst.n_segments)] if lst.speech_index else None
    out = []
    for i in range(lst.n_segments):
        s = lst.segments[i]
        words = None
        if s.words:
            words = [WordTimestamp(s.words[k].text.decode("utf-8", "replace"), s.words[k].start, s.words[k].end,
                                   s.words[k].probability if s.words[k].has_probability else None)
                     for k in range(s.n_words)]
        out.append(Segment(s.start, s.end, s.text.decode("utf-8", "replace"), words,
                           s.speaker_id.decode() if s.speaker_id else None))
    lang = lst.detected_lang.decode() if lst.detected_lang else None
    L.load().wdr_segment_list_free(lst_ptr)
    return (out, lang, index) if with_index else (out, lang)


def _callbacks(cb: Optional[Callbacks], keep: _Keep):
    if cb is None:
        return None
    c = L.Callbacks()
    if cb.progress:
        c.progress = keep(L.PROGRESS_FN(lambda u, p, t, lbl: cb.progress(int(p), ProgressType(t), lbl.decode())))
    if cb.new_segment_callback:
        def seg_cb(u, sp):
            s = sp.contents
            words = None
            if s.words:
                words = [WordTimestamp(s.words[k].text.decode(), s.words[k].start, s.words[k].end,
                                       s.words[k].probability if s.words[k].has_probability else None)
                         for k in range(s.n_words)]
            cb.new_segment_callback(Segment(s.start, s.end, s.text.decode(), words,
                                            s.speaker_id.decode() if s.speaker_id else None))
        c.new_segment = keep(L.SEGMENT_FN(seg_cb))
    if cb.is_cancelled:
        c.is_cancelled = keep(L.CANCEL_FN(lambda u: 1 if cb.is_cancelled() else 0))
    return keep(c)


def read_wav(path: str) -> np.ndarray:
    """audio::read_wav (src/audio.rs:4-24)."""
    lib = L.load()
    p = C.POINTER(C.c_int16)()
    n = C.c_size_t()
    L.check(lib.wdr_read_wav(path.encode(), C.byref(p), C.byref(n)))
    out = np.ctypeslib.as_array(p, shape=(n.value,)).copy() if n.value else np.zeros(0, np.int16)
    lib.wdr_free(p)
    return out


def vad_merge(segs_cs, samples: np.ndarray):
    """The crate's own post-processing of whisper.cpp VAD segments (src/vad.rs:33-84)."""
    lib = L.load()
    st = np.ascontiguousarray([s for s, _ in segs_cs], np.float64)
    en = np.ascontiguousarray([e for _, e in segs_cs], np.float64)
    n = len(st)
    mask = np.zeros(2 * max(n, 1))
    merged = np.zeros(2 * max(n, 1))
    idx = np.zeros(2 * max(n, 1), np.int64)
    nm, nmr = C.c_size_t(), C.c_size_t()
    smp = np.ascontiguousarray(samples, np.int16)
    L.check(lib.wdr_vad_merge(st.ctypes.data_as(C.POINTER(C.c_double)), en.ctypes.data_as(C.POINTER(C.c_double)), n,
                              smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size,
                              mask.ctypes.data_as(C.POINTER(C.c_double)), C.byref(nm),
                              merged.ctypes.data_as(C.POINTER(C.c_double)), idx.ctypes.data_as(C.POINTER(C.c_int64)),
                              C.byref(nmr)))
    m = [(mask[2 * i], mask[2 * i + 1]) for i in range(nm.value)]
    out = [SpeechSegment(merged[2 * i], merged[2 * i + 1], smp[idx[2 * i]:idx[2 * i + 1]].copy())
           for i in range(nmr.value)]
    return m, out


def vad_segments_from_probs(probs) -> list:
    """whisper.cpp whisper_vad_segments_from_probs with the reference's VAD params
    (src/vad.rs:21-22): [(start_cs, end_cs)] as f32 values."""
    lib = L.load()
    p = np.ascontiguousarray(probs, np.float32)
    out = np.zeros(2 * max(1, p.size), np.float32)
    n = C.c_size_t()
    L.check(lib.wdr_vad_segments_from_probs(p.ctypes.data_as(C.POINTER(C.c_float)), p.size,
                                            out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(n)))
    return [(float(out[2 * i]), float(out[2 * i + 1])) for i in range(n.value)]


class Vad:
    """Silero VAD on the GPU (src/vad.rs:6-85).  model_path: whisper.cpp's ggml-silero-v5.1.2.bin;
    None = synthetic seeded weights."""

    def __init__(self, model_path: Optional[str] = None, gpu_device: Optional[int] = None):
        self._lib = L.load()
        h = C.c_void_p()
        L.check(self._lib.wdr_vad_create(_s(model_path), 0 if gpu_device is None else 1, gpu_device or 0, C.byref(h)))
        self.h = h
        self.last_us_per_step = 0.0

    def probs(self, samples: np.ndarray) -> np.ndarray:
        smp = np.ascontiguousarray(samples, np.int16)
        out = np.zeros((smp.size + 511) // 512, np.float32)
        us = C.c_double()
        L.check(self._lib.wdr_vad_probs(self.h, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size,
                                        out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(us)))
        self.last_us_per_step = us.value
        return out

    def get_segments(self, samples: np.ndarray, materialize: bool = True):
        """-> (mask [(start_s, end_s)], [SpeechSegment]) exactly as vad::get_segments.
        materialize=False returns only the segment (start, end) pairs (no sample copies)."""
        smp = np.ascontiguousarray(samples, np.int16)
        mp, nm = C.POINTER(C.c_double)(), C.c_size_t()
        sp, ns = C.POINTER(L.SpeechSegment)(), C.c_size_t()
        L.check(self._lib.wdr_vad_get_segments(self.h, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size,
                                               C.byref(mp), C.byref(nm), C.byref(sp), C.byref(ns)))
        us = C.c_double()
        L.check(self._lib.wdr_vad_stats(self.h, C.byref(us)))
        self.last_us_per_step = us.value
        try:
            mask = [(mp[2 * i], mp[2 * i + 1]) for i in range(nm.value)]
            base = smp.ctypes.data
            segs = []
            for i in range(ns.value):
                s = sp[i]
                if not materialize:
                    segs.append((s.start, s.end))
                    continue
                off = (C.cast(s.samples, C.c_void_p).value - base) // 2
                segs.append(SpeechSegment(s.start, s.end, smp[off:off + s.n_samples].copy()))
        finally:
            self._lib.wdr_free(C.cast(mp, C.c_void_p))
            self._lib.wdr_free(C.cast(sp, C.c_void_p))
        return mask, segs

    def close(self):
        if self.h:
            self._lib.wdr_vad_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SpeakerManager:
    """pyannote_rs::EmbeddingManager as the reference drives it (src/transcribe.rs:478-497)."""

    def __init__(self, max_speakers: Optional[int] = None):
        self._lib = L.load()
        h = C.c_void_p()
        L.check(self._lib.wdr_speakers_new(0 if max_speakers is None else 1, max_speakers or 0, C.byref(h)))
        self.h = h

    def assign(self, emb, threshold: float = 0.5) -> str:
        buf = C.create_string_buffer(32)
        if emb is None:
            L.check(self._lib.wdr_speakers_assign(self.h, None, 0, threshold, buf, 32))
        else:
            e = np.ascontiguousarray(emb, np.float32)
            L.check(self._lib.wdr_speakers_assign(self.h, e.ctypes.data_as(C.POINTER(C.c_float)), e.size, threshold,
                                                  buf, 32))
        return buf.value.decode()

    def __del__(self):
        try:
            self._lib.wdr_speakers_free(self.h)
        except Exception:
            pass


class Diarizer:
    """pyannote segmentation-3.0 + CAM++ on the GPU (src/engine.rs:89-122,
    src/transcribe.rs:461-497).  Model paths: the ONNX files; None = synthetic seeded weights."""

    def __init__(self, gpu_device: Optional[int] = None, segment_model_path: Optional[str] = None,
                 embedding_model_path: Optional[str] = None):
        self._lib = L.load()
        h = C.c_void_p()
        L.check(self._lib.wdr_diarizer_create(_s(segment_model_path), _s(embedding_model_path),
                                              0 if gpu_device is None else 1, gpu_device or 0, C.byref(h)))
        self.h = h

    def frame_classes(self, samples: np.ndarray, logprobs: bool = False):
        smp = np.ascontiguousarray(samples, np.int16)
        nw = smp.size // 160000 + 1
        cls = np.zeros(nw * 589, np.int32)
        lp = np.zeros(nw * 589 * 7, np.float32) if logprobs else None
        L.check(self._lib.wdr_diarize_frame_classes(self.h, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size,
                                                    cls.ctypes.data_as(C.POINTER(C.c_int32)),
                                                    lp.ctypes.data_as(C.POINTER(C.c_float)) if logprobs else None))
        cls = cls.reshape(nw, 589)
        return (cls, lp.reshape(nw, 589, 7)) if logprobs else cls

    def get_segments(self, samples: np.ndarray, materialize: bool = True):
        """pyannote_rs::get_segments (wdr_diarize_get_segments: the segments and their samples are
        made in libwdr).  materialize=False returns (start, end) pairs without copying every
        segment's samples a second time into Python arrays (as Vad.get_segments)."""
        smp = np.ascontiguousarray(samples, np.int16)
        sp, ns = C.POINTER(L.SpeechSegment)(), C.c_size_t()
        L.check(self._lib.wdr_diarize_get_segments(self.h, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size,
                                                   C.byref(sp), C.byref(ns)))
        try:
            if not materialize:
                return [(sp[i].start, sp[i].end) for i in range(ns.value)]
            return [SpeechSegment(sp[i].start, sp[i].end, np.ctypeslib.as_array(sp[i].samples, (sp[i].n_samples,)).copy()
                                  if sp[i].n_samples else np.zeros(0, np.int16)) for i in range(ns.value)]
        finally:
            self._lib.wdr_free(C.cast(sp, C.c_void_p))

    @staticmethod
    def segments_from_classes(cls: np.ndarray, samples: np.ndarray):
        """pyannote_rs::get_segments' stitching of frame classes [n/160000 + 1][589] computed
        elsewhere (window shards of several GPUs)."""
        smp = np.ascontiguousarray(samples, np.int16)
        c = np.ascontiguousarray(cls, np.int32)
        sp, ns = C.POINTER(L.SpeechSegment)(), C.c_size_t()
        lib = L.load()
        L.check(lib.wdr_diarize_segments_from_classes(c.ctypes.data_as(C.POINTER(C.c_int32)), c.shape[0],
                                                      smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size,
                                                      C.byref(sp), C.byref(ns)))
        try:
            return [SpeechSegment(sp[i].start, sp[i].end, np.ctypeslib.as_array(sp[i].samples, (sp[i].n_samples,)).copy()
                                  if sp[i].n_samples else np.zeros(0, np.int16)) for i in range(ns.value)]
        finally:
            lib.wdr_free(C.cast(sp, C.c_void_p))

    def fbank(self, samples: np.ndarray) -> np.ndarray:
        smp = np.ascontiguousarray(samples, np.int16)
        out = np.zeros((smp.size // 160 + 1, 80), np.float32)
        nf = C.c_size_t()
        L.check(self._lib.wdr_diarize_fbank(self.h, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size,
                                            out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(nf)))
        return out[:nf.value]

    def embedding(self, samples: np.ndarray):
        smp = np.ascontiguousarray(samples, np.int16)
        out = np.zeros(512, np.float32)
        ok = C.c_int8()
        L.check(self._lib.wdr_diarize_embedding(self.h, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size,
                                                out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(ok)))
        return out if ok.value else None

    def embedding_batch(self, segments):
        """Embeddings of several utterances in one batched forward (wdr_diarize_embedding_batch):
        a list with None where embedding() would return None."""
        smp = [np.ascontiguousarray(x, np.int16) for x in segments]
        B = len(smp)
        ptrs = (C.POINTER(C.c_int16) * max(B, 1))(*[x.ctypes.data_as(C.POINTER(C.c_int16)) for x in smp])
        ns = (C.c_size_t * max(B, 1))(*[x.size for x in smp])
        out = np.zeros((max(B, 1), 512), np.float32)
        ok = (C.c_int8 * max(B, 1))()
        L.check(self._lib.wdr_diarize_embedding_batch(self.h, ptrs, ns, B, out.ctypes.data_as(C.POINTER(C.c_float)), ok))
        return [out[b].copy() if ok[b] else None for b in range(B)]

    def stats(self):
        a, b = C.c_double(), C.c_double()
        L.check(self._lib.wdr_diarize_stats(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def __del__(self):
        try:
            self._lib.wdr_diarizer_free(self.h)
        except Exception:
            pass


def model_file_tensors(kind: str, path: str) -> dict:
    """Tensors of a VAD / diarization model file as libwdr's loader maps them (oracle names):
    kind 'silero' (whisper.cpp ggml), 'segmentation' / 'campplus' (ONNX).  Host only."""
    lib = L.load()
    k = {"silero": 0, "segmentation": 1, "campplus": 2}[kind]
    names, data, n = C.c_void_p(), C.POINTER(C.c_float)(), C.c_size_t()
    L.check(lib.wdr_dbg_model_file(k, path.encode(), C.byref(names), C.byref(data), C.byref(n)))
    try:
        txt = C.cast(names, C.c_char_p).value.decode()
        flat = np.ctypeslib.as_array(data, (max(1, n.value),))[:n.value].copy()
    finally:
        lib.wdr_free(names)
        lib.wdr_free(C.cast(data, C.c_void_p))
    out, o = {}, 0
    for line in txt.splitlines():
        name, cnt = line.rsplit(":", 1)
        out[name] = flat[o:o + int(cnt)]
        o += int(cnt)
    return out


def ggml_info(path: str) -> dict:
    """Header of a whisper.cpp ggml model file (wdr_ggml_info; parses the whole file, no GPU)."""
    lib = L.load()
    hp = (C.c_int32 * 11)()
    nt, nv = C.c_int64(), C.c_int64()
    L.check(lib.wdr_ggml_info(path.encode(), hp, C.byref(nt), C.byref(nv)))
    keys = ["n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer", "n_text_ctx",
            "n_text_state", "n_text_head", "n_text_layer", "n_mels", "ftype"]
    return {**dict(zip(keys, list(hp))), "n_tensors": nt.value, "n_vocab_tokens": nv.value}


class WhisperContext:
    """transcribe::create_context (src/transcribe.rs:89-166) + its whisper_state."""

    def __init__(self, model_name: str, model_path: Optional[str] = None, gpu_device: Optional[int] = None,
                 use_gpu: Optional[bool] = None, enable_dtw: Optional[bool] = True,
                 enable_flash_attn: Optional[bool] = None, num_samples: Optional[int] = None,
                 synthetic: Optional[Synthetic] = None):
        lib = L.load()
        self._lib = lib
        h = C.c_void_p()
        syn = _syn(synthetic)
        L.check(lib.wdr_context_create(_s(model_path), model_name.encode(), 0 if gpu_device is None else 1,
                                       gpu_device or 0, _ob(use_gpu), _ob(enable_dtw), _ob(enable_flash_attn),
                                       0 if num_samples is None else 1, num_samples or 0,
                                       C.byref(syn) if syn else None, C.byref(h)))
        self.h = h
        self.synthetic = synthetic
        hp = (C.c_int32 * 10)()
        L.check(lib.wdr_context_hparams(h, hp))
        keys = ["n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer", "n_text_ctx",
                "n_text_state", "n_text_head", "n_text_layer", "n_mels"]
        self.hparams = dict(zip(keys, list(hp)))

    def close(self):
        if self.h:
            self._lib.wdr_context_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- run_transcription_pipeline (src/transcribe.rs:323-535)
    def run_pipeline(self, speech_segments, options: TranscribeOptions, callbacks: Optional[Callbacks] = None,
                     synthetic: Optional[Synthetic] = None, with_index: bool = False,
                     diarize_options: Optional[DiarizeOptions] = None):
        """transcribe::run_transcription_pipeline(ctx, segments, options, diarize_options, ...)
        -> (segments, detected_lang) [+ the input SpeechSegment index of every output segment
        when with_index].  Speakers are assigned iff diarize_options is given (as the
        reference's Option<DiarizeOptions>)."""
        keep = _Keep()
        arr = (L.SpeechSegment * max(1, len(speech_segments)))()
        for i, s in enumerate(speech_segments):
            smp = keep(np.ascontiguousarray(s.samples, np.int16))
            arr[i] = L.SpeechSegment(s.start, s.end, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size)
        out = C.POINTER(L.SegmentList)()
        syn = _syn(synthetic or self.synthetic)
        d = _dopts(diarize_options, keep)
        L.check(self._lib.wdr_run_pipeline(self.h, arr, len(speech_segments), _opts(options, keep),
                                           C.byref(d) if d is not None else None,
                                           C.byref(syn) if syn else None, _callbacks(callbacks, keep),
                                           C.byref(out)))
        return _segments(out, with_index)

    def run_pipeline_raw(self, speech_segments, options: TranscribeOptions, synthetic: Optional[Synthetic] = None):
        """run_pipeline without the cross-segment overlap clip and speaker assignment
        (wdr_run_pipeline_raw): (segments, detected_lang, speech index per segment)."""
        keep = _Keep()
        arr = (L.SpeechSegment * max(1, len(speech_segments)))()
        for i, s in enumerate(speech_segments):
            smp = keep(np.ascontiguousarray(s.samples, np.int16))
            arr[i] = L.SpeechSegment(s.start, s.end, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size)
        out = C.POINTER(L.SegmentList)()
        syn = _syn(synthetic or self.synthetic)
        L.check(self._lib.wdr_run_pipeline_raw(self.h, arr, len(speech_segments), _opts(options, keep),
                                               C.byref(syn) if syn else None, C.byref(out)))
        segs, lang, index = _segments(out, True)
        return segs, lang, index or []

    def run_pipeline_block(self, speech_segments, options: TranscribeOptions, rng_in: Optional[str] = None,
                           synthetic: Optional[Synthetic] = None):
        """run_pipeline_raw continuing decoder 0's RNG stream (wdr_run_pipeline_block):
        (segments, detected_lang, speech index per segment, sampled flag per speech segment,
        rng state after the block)."""
        keep = _Keep()
        arr = (L.SpeechSegment * max(1, len(speech_segments)))()
        for i, s in enumerate(speech_segments):
            smp = keep(np.ascontiguousarray(s.samples, np.int16))
            arr[i] = L.SpeechSegment(s.start, s.end, smp.ctypes.data_as(C.POINTER(C.c_int16)), smp.size)
        out = C.POINTER(L.SegmentList)()
        syn = _syn(synthetic or self.synthetic)
        sampled = (C.c_int8 * max(1, len(speech_segments)))()
        rng = C.c_void_p()
        L.check(self._lib.wdr_run_pipeline_block(self.h, arr, len(speech_segments), _opts(options, keep),
                                                 C.byref(syn) if syn else None, _s(rng_in), sampled, C.byref(rng),
                                                 C.byref(out)))
        rng_out = C.cast(rng, C.c_char_p).value.decode()
        self._lib.wdr_free(rng)
        segs, lang, index = _segments(out, True)
        return segs, lang, index or [], [bool(sampled[i]) for i in range(len(speech_segments))], rng_out

    @property
    def devices(self) -> List[int]:
        """GPU ordinals this context runs on (wdr_context_devices): gpu_device=None -> every
        visible GPU, the decode chains spread over them."""
        n = C.c_int32()
        ids = (C.c_int32 * 8)()
        L.check(self._lib.wdr_context_devices(self.h, C.byref(n), ids, 8))
        return [ids[i] for i in range(min(n.value, 8))]

    def set_encoder_fp8(self, on: bool):
        """fp8 (e4m3) encoder GEMMs, BASELINE configs[4] (wdr_context_set_encoder_fp8)."""
        L.check(self._lib.wdr_context_set_encoder_fp8(self.h, 1 if on else 0))

    def set_chains(self, n: int):
        """Decode chains per GPU for run_pipeline calls (wdr_context_set_chains): n blocks of the
        speech segments per GPU decoded concurrently with batched steps, exact prompt fix-up."""
        L.check(self._lib.wdr_context_set_chains(self.h, int(n)))

    def set_early_fixup(self, mode: int):
        """Test seam (wdr_dbg_set_early_fixup): 0 off, 1 after the predecessor finished, 2 forced
        (wait for the predecessor to finish), 3 from the predecessor's speculative prompt (the
        default), -1 env default."""
        L.check(self._lib.wdr_dbg_set_early_fixup(self.h, int(mode)))

    def stage_times(self) -> dict:
        t = L.StageTimes()
        L.check(self._lib.wdr_context_stage_times(self.h, C.byref(t)))
        return {f: getattr(t, f) for f, _ in L.StageTimes._fields_}

    # -- test seams
    def state_full(self, samples_f32: np.ndarray, options: TranscribeOptions, initial_prompt: Optional[str] = None,
                   synthetic: Optional[Synthetic] = None):
        keep = _Keep()
        x = np.ascontiguousarray(samples_f32, np.float32)
        segs = C.POINTER(L.ResultSeg)()
        n = C.c_size_t()
        lang = C.c_int32()
        syn = _syn(synthetic or self.synthetic)
        L.check(self._lib.wdr_state_full(self.h, x.ctypes.data_as(C.POINTER(C.c_float)), x.size, _opts(options, keep),
                                         C.byref(syn) if syn else None, _s(initial_prompt), C.byref(segs), C.byref(n),
                                         C.byref(lang)))
        out = []
        for i in range(n.value):
            s = segs[i]
            toks = [dict(id=t.id, tid=t.tid, p=t.p, plog=t.plog, pt=t.pt, ptsum=t.ptsum, t0=t.t0, t1=t.t1,
                         t_dtw=t.t_dtw) for t in (s.tokens[k] for k in range(s.n_tokens))]
            out.append(dict(t0=s.t0, t1=s.t1, text=s.text.decode(), tokens=toks))
        self._lib.wdr_result_free(segs, n.value)
        return out, lang.value

    def log_mel_window(self, x: np.ndarray, seek: int = 0) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float32)
        out = np.zeros((self.hparams["n_mels"], 3000), np.float32)
        L.check(self._lib.wdr_dbg_log_mel(self.h, x.ctypes.data_as(C.POINTER(C.c_float)), x.size, seek,
                                          out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def encode(self, mel_window: np.ndarray) -> np.ndarray:
        m = np.ascontiguousarray(mel_window, np.float32)
        out = np.zeros((1500, self.hparams["n_audio_state"]), np.float32)
        L.check(self._lib.wdr_dbg_encode(self.h, m.ctypes.data_as(C.POINTER(C.c_float)),
                                         out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def cross_kv(self) -> np.ndarray:
        """Cross K/V of the last encode() window: [1500][n_text_layer][2][d]."""
        h = self.hparams
        out = np.zeros((1500, h["n_text_layer"], 2, h["n_text_state"]), np.float32)
        L.check(self._lib.wdr_dbg_cross_kv(self.h, out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def decode(self, tokens) -> np.ndarray:
        t = np.ascontiguousarray(tokens, np.int32)
        out = np.zeros(self.hparams["n_vocab"], np.float32)
        L.check(self._lib.wdr_dbg_decode(self.h, t.ctypes.data_as(C.POINTER(C.c_int32)), t.size,
                                         out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def step(self, tokens) -> np.ndarray:
        """Prefill tokens[:-1], then one decode step of tokens[-1]: the step's logits."""
        t = np.ascontiguousarray(tokens, np.int32)
        out = np.zeros(self.hparams["n_vocab"], np.float32)
        L.check(self._lib.wdr_dbg_step(self.h, t.ctypes.data_as(C.POINTER(C.c_int32)), t.size,
                                       out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def logit_rules(self, logits, ctls, temps=None, max_initial_ts: float = 1.0, suppress_blank: bool = True):
        """whisper.cpp's logit rules + greedy pick on the GPU (wdr_dbg_logits): logits [R][n_vocab],
        ctls = R dicts of n_tokens / last_ts / pen_ts / has_ts / seek_delta / force_kind / force_tok.
        Returns R dicts: id, tid, p, plog, pt, ptsum, nosp."""
        lg = np.ascontiguousarray(logits, np.float32)
        R = lg.shape[0]
        keys = ("n_tokens", "last_ts", "pen_ts", "has_ts", "seek_delta", "force_kind", "force_tok")
        ctl = np.ascontiguousarray([[int(c.get(k, 0)) for k in keys] for c in ctls], np.int32)
        tt = np.ascontiguousarray(temps if temps is not None else [0.0] * R, np.float32)
        ids = np.zeros((R, 2), np.int32)
        f = np.zeros((R, 5), np.float32)
        L.check(self._lib.wdr_dbg_logits(self.h, lg.ctypes.data_as(C.POINTER(C.c_float)), R,
                                         ctl.ctypes.data_as(C.POINTER(C.c_int32)),
                                         tt.ctypes.data_as(C.POINTER(C.c_float)), float(max_initial_ts),
                                         1 if suppress_blank else 0, ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                         f.ctypes.data_as(C.POINTER(C.c_float))))
        return [dict(id=int(ids[r, 0]), tid=int(ids[r, 1]), p=float(f[r, 0]), plog=float(f[r, 1]), pt=float(f[r, 2]),
                     ptsum=float(f[r, 3]), nosp=float(f[r, 4])) for r in range(R)]

    def batch_step_ms(self, tokens, rows: int, iters: int = 50) -> float:
        """Host ms per multi-chain batched step of `rows` rows on the last encoded window
        (wdr_dbg_batch_step probe seam)."""
        t = np.ascontiguousarray(tokens, np.int32)
        ms = C.c_double()
        L.check(self._lib.wdr_dbg_batch_step(self.h, t.ctypes.data_as(C.POINTER(C.c_int32)), t.size, int(rows),
                                             int(iters), C.byref(ms)))
        return ms.value

    def capture(self, tokens, n_aheads: int) -> np.ndarray:
        t = np.ascontiguousarray(tokens, np.int32)
        out = np.zeros((n_aheads, t.size, 1500), np.float32)
        L.check(self._lib.wdr_dbg_capture(self.h, t.ctypes.data_as(C.POINTER(C.c_int32)), t.size,
                                          out.ctypes.data_as(C.POINTER(C.c_float))))
        return out


class Engine:
    """Engine (src/engine.rs:52-217)."""

    def __init__(self, cfg: Optional[EngineConfig] = None, synthetic: Optional[Synthetic] = None):
        cfg = cfg or EngineConfig()
        lib = L.load()
        self._lib = lib
        self._keep = _Keep()
        c = L.EngineConfig(self._keep(_s(cfg.cache_dir)), _ob(cfg.enable_dtw), _ob(cfg.enable_flash_attn),
                           _ob(cfg.use_gpu), 0 if cfg.gpu_device is None else 1, cfg.gpu_device or 0,
                           self._keep(_s(cfg.vad_model_path)), self._keep(_s(cfg.diarize_segment_model_path)),
                           self._keep(_s(cfg.diarize_embedding_model_path)))
        h = C.c_void_p()
        L.check(lib.wdr_engine_new(C.byref(c), C.byref(h)))
        self.h = h
        if synthetic is not None:
            s = _syn(synthetic)
            L.check(lib.wdr_engine_set_synthetic(h, C.byref(s)))

    def transcribe_audio(self, audio_path: str, options: TranscribeOptions,
                         formatting_overrides=None, cb: Optional[Callbacks] = None) -> List[Segment]:
        keep = _Keep()
        out = C.POINTER(L.SegmentList)()
        ov = _fmt(formatting_overrides)
        L.check(self._lib.wdr_transcribe_audio(self.h, audio_path.encode(), _opts(options, keep),
                                               C.byref(ov) if ov is not None else None,
                                               _callbacks(cb, keep), C.byref(out)))
        segs, _ = _segments(out)
        return segs

    def close(self):
        if self.h:
            self._lib.wdr_engine_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
