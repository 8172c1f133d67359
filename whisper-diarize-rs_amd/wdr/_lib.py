"""ctypes binding of libwdr (include/wdr.h).  Loads the in-tree libwdr.so built by
`__graft_entry__.build()` / `make -C whisper-diarize-rs_amd`; fails loudly if it is missing
(there is no CPU fallback: the CPU restatement under oracle/ is test-only)."""
from __future__ import annotations

import atexit
import ctypes as C
import os
import re

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# WDR_AB_LIB: another build of libwdr for same-box A/B runs (tools/ab_env.sh); unset = in-tree
LIB_PATH = os.environ.get("WDR_AB_LIB") or os.path.join(PKG_DIR, "libwdr.so")
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "wdr.h")

i8, i32, i64, u64 = C.c_int8, C.c_int32, C.c_int64, C.c_uint64
f32, f64, cstr, vp, sz = C.c_float, C.c_double, C.c_char_p, C.c_void_p, C.c_size_t


class EngineConfig(C.Structure):
    _fields_ = [("cache_dir", cstr), ("enable_dtw", i8), ("enable_flash_attn", i8), ("use_gpu", i8),
                ("has_gpu_device", i8), ("gpu_device", i32), ("vad_model_path", cstr),
                ("diarize_segment_model_path", cstr), ("diarize_embedding_model_path", cstr)]


class Advanced(C.Structure):
    _fields_ = [("sampling_strategy", cstr), ("has_best_of_or_beam_size", i8), ("best_of_or_beam_size", i32),
                ("has_n_threads", i8), ("n_threads", i32), ("has_temperature", i8), ("temperature", f32),
                ("has_max_text_ctx", i8), ("max_text_ctx", i32), ("init_prompt", cstr),
                ("has_diarize_threshold", i8), ("diarize_threshold", f32)]


class TranscribeOptions(C.Structure):
    _fields_ = [("has_offset", i8), ("offset", f64), ("model", cstr), ("lang", cstr), ("whisper_to_english", i8),
                ("translate_target", cstr), ("enable_vad", i8), ("enable_diarize", i8), ("has_max_speakers", i8),
                ("max_speakers", u64), ("advanced", C.POINTER(Advanced))]


class DiarizeOptions(C.Structure):
    _fields_ = [("segment_model_path", cstr), ("embedding_model_path", cstr), ("threshold", f32),
                ("max_speakers", u64)]


class Synthetic(C.Structure):
    _fields_ = [("weight_std", f64), ("emb_std", f64), ("force_len_rate", f32), ("disable_fallback", i8)]


class FormattingOverrides(C.Structure):
    _fields_ = [("has_max_chars_per_line", i8), ("max_chars_per_line", u64), ("has_max_lines", i8),
                ("max_lines", u64), ("has_cps_cap", i8), ("cps_cap", f64), ("has_split_gap_sec", i8),
                ("split_gap_sec", f64), ("has_comma_min_chars_before_allow", i8),
                ("comma_min_chars_before_allow", u64), ("has_min_word_dur", i8), ("min_word_dur", f64),
                ("has_min_sub_dur", i8), ("min_sub_dur", f64), ("has_max_sub_dur", i8), ("max_sub_dur", f64),
                ("has_soft_max_words_per_line", i8), ("soft_max_words_per_line", u64),
                ("insert_interword_space", i8), ("use_grapheme_len", i8), ("enforce_kinsoku", i8),
                ("allow_comma_split", i8)]


class Word(C.Structure):
    _fields_ = [("text", cstr), ("start", f64), ("end", f64), ("has_probability", i8), ("probability", f32)]


class Segment(C.Structure):
    _fields_ = [("start", f64), ("end", f64), ("text", cstr), ("words", C.POINTER(Word)), ("n_words", sz),
                ("speaker_id", cstr)]


class SegmentList(C.Structure):
    _fields_ = [("segments", C.POINTER(Segment)), ("n_segments", sz), ("detected_lang", cstr),
                ("speech_index", C.POINTER(C.c_int64))]


class SpeechSegment(C.Structure):
    _fields_ = [("start", f64), ("end", f64), ("samples", C.POINTER(C.c_int16)), ("n_samples", sz)]


PROGRESS_FN = C.CFUNCTYPE(None, vp, i32, i32, cstr)
SEGMENT_FN = C.CFUNCTYPE(None, vp, C.POINTER(Segment))
CANCEL_FN = C.CFUNCTYPE(C.c_int, vp)


class Callbacks(C.Structure):
    _fields_ = [("user", vp), ("progress", PROGRESS_FN), ("new_segment", SEGMENT_FN), ("is_cancelled", CANCEL_FN)]


class StageTimes(C.Structure):
    _fields_ = [("mel", f64), ("encode", f64), ("decode", f64), ("dtw", f64), ("vad", f64), ("total", f64),
                ("windows", i64), ("decode_steps", i64), ("prefills", i64), ("lang", f64), ("prompt_gpu", f64),
                ("embed", f64), ("chains", i64), ("batch_launches", i64), ("batch_rows", i64),
                ("fixup_segments", i64), ("replay_segments", i64), ("spec_s", f64), ("fixup_s", f64),
                ("batch_step_s", f64), ("early_fixup_segments", i64), ("batch_prefill_rows", i64),
                ("batch_dtw_rows", i64), ("batch_prefills", i64), ("batch_dtws", i64), ("batch_mixed", i64),
                ("batch_xattn_groups", i64), ("batch_xattn_tiles", i64), ("dtwq_passes", i64), ("dtwq_rows", i64),
                ("dtwq_jobs", i64), ("lang_passes", i64), ("lang_rows", i64)]


class Token(C.Structure):
    _fields_ = [("id", i32), ("tid", i32), ("p", f32), ("plog", f32), ("pt", f32), ("ptsum", f32),
                ("t0", i64), ("t1", i64), ("t_dtw", i64)]


class ResultSeg(C.Structure):
    _fields_ = [("t0", i64), ("t1", i64), ("text", cstr), ("tokens", C.POINTER(Token)), ("n_tokens", sz)]


P = C.POINTER
_SIGS = {
    "wdr_last_error": (cstr, []),
    "wdr_abi_version": (C.c_int, []),
    "wdr_device_count": (C.c_int, []),
    "wdr_shutdown": (None, []),
    "wdr_engine_new": (C.c_int, [P(EngineConfig), P(vp)]),
    "wdr_engine_free": (None, [vp]),
    "wdr_engine_set_synthetic": (C.c_int, [vp, P(Synthetic)]),
    "wdr_transcribe_audio": (C.c_int, [vp, cstr, P(TranscribeOptions), P(FormattingOverrides), P(Callbacks),
                                       P(P(SegmentList))]),
    "wdr_read_wav": (C.c_int, [cstr, P(P(C.c_int16)), P(sz)]),
    "wdr_dbg_model_file": (C.c_int, [i32, cstr, P(C.c_void_p), P(P(f32)), P(sz)]),
    "wdr_process_segments": (C.c_int, [P(Segment), sz, cstr, P(FormattingOverrides), i8, P(f64), sz,
                                       P(P(SegmentList))]),
    "wdr_free": (None, [vp]),
    "wdr_vad_merge": (C.c_int, [P(f64), P(f64), sz, P(C.c_int16), sz, P(f64), P(sz), P(f64), P(i64), P(sz)]),
    "wdr_vad_create": (C.c_int, [cstr, i8, i32, P(vp)]),
    "wdr_vad_free": (None, [vp]),
    "wdr_vad_probs": (C.c_int, [vp, P(C.c_int16), sz, P(f32), P(f64)]),
    "wdr_vad_stats": (C.c_int, [vp, P(f64)]),
    "wdr_vad_segments_from_probs": (C.c_int, [P(f32), sz, P(f32), P(sz)]),
    "wdr_vad_get_segments": (C.c_int, [vp, P(C.c_int16), sz, P(P(f64)), P(sz), P(P(SpeechSegment)), P(sz)]),
    "wdr_diarizer_create": (C.c_int, [cstr, cstr, i8, i32, P(vp)]),
    "wdr_diarizer_free": (None, [vp]),
    "wdr_diarize_frame_classes": (C.c_int, [vp, P(C.c_int16), sz, P(i32), P(f32)]),
    "wdr_diarize_get_segments": (C.c_int, [vp, P(C.c_int16), sz, P(P(SpeechSegment)), P(sz)]),
    "wdr_diarize_segments_from_classes": (C.c_int, [P(i32), sz, P(C.c_int16), sz, P(P(SpeechSegment)), P(sz)]),
    "wdr_diarize_fbank": (C.c_int, [vp, P(C.c_int16), sz, P(f32), P(sz)]),
    "wdr_diarize_embedding": (C.c_int, [vp, P(C.c_int16), sz, P(f32), P(i8)]),
    "wdr_diarize_embedding_batch": (C.c_int, [vp, P(P(C.c_int16)), P(sz), i32, P(f32), P(i8)]),
    "wdr_diarize_stats": (C.c_int, [vp, P(f64), P(f64)]),
    "wdr_speakers_new": (C.c_int, [i8, u64, P(vp)]),
    "wdr_speakers_free": (None, [vp]),
    "wdr_speakers_assign": (C.c_int, [vp, P(f32), i32, f32, C.c_char_p, sz]),
    "wdr_context_create": (C.c_int, [cstr, cstr, i8, i32, i8, i8, i8, i8, u64, P(Synthetic), P(vp)]),
    "wdr_context_free": (None, [vp]),
    "wdr_run_pipeline_raw": (C.c_int, [vp, P(SpeechSegment), sz, P(TranscribeOptions), P(Synthetic),
                                       P(P(SegmentList))]),
    "wdr_run_pipeline": (C.c_int, [vp, P(SpeechSegment), sz, P(TranscribeOptions), P(DiarizeOptions), P(Synthetic),
                                   P(Callbacks), P(P(SegmentList))]),
    "wdr_run_pipeline_block": (C.c_int, [vp, P(SpeechSegment), sz, P(TranscribeOptions), P(Synthetic), cstr, P(i8),
                                         P(C.c_void_p), P(P(SegmentList))]),
    "wdr_segment_list_free": (None, [P(SegmentList)]),
    "wdr_context_set_chains": (C.c_int, [vp, i32]),
    "wdr_context_devices": (C.c_int, [vp, P(i32), P(i32), i32]),
    "wdr_context_set_encoder_fp8": (C.c_int, [vp, C.c_int8]),
    "wdr_dbg_set_early_fixup": (C.c_int, [vp, i32]),
    "wdr_dbg_set_gemm32": (C.c_int, [i32]),
    "wdr_ggml_info": (C.c_int, [cstr, P(i32), P(i64), P(i64)]),
    "wdr_dbg_batch_step": (C.c_int, [vp, P(i32), sz, i32, i32, P(f64)]),
    "wdr_context_stage_times": (C.c_int, [vp, P(StageTimes)]),
    "wdr_context_hparams": (C.c_int, [vp, P(i32)]),
    "wdr_prof_set": (C.c_int, [i32]),
    "wdr_prof_read": (C.c_int, [P(f64), P(i64), P(f64), P(f64)]),
    "wdr_prof_set_mask": (C.c_int, [i32]),
    "wdr_prof_read_class": (C.c_int, [i32, P(f64), P(i64), P(f64), P(f64)]),
    "wdr_prof_read_clock": (C.c_int, [i32, P(f64), P(i64), P(f64), P(f64)]),
    "wdr_state_full": (C.c_int, [vp, P(f32), sz, P(TranscribeOptions), P(Synthetic), cstr, P(P(ResultSeg)), P(sz),
                                 P(i32)]),
    "wdr_result_free": (None, [P(ResultSeg), sz]),
    "wdr_dbg_log_mel": (C.c_int, [vp, P(f32), sz, i32, P(f32)]),
    "wdr_dbg_energy": (C.c_int, [P(f32), sz, P(f32)]),
    "wdr_dbg_mfma_scale": (C.c_int, [P(C.c_uint8), P(C.c_uint8), P(i32), P(i32), P(f32)]),
    "wdr_dbg_encode": (C.c_int, [vp, P(f32), P(f32)]),
    "wdr_dbg_decode": (C.c_int, [vp, P(i32), sz, P(f32)]),
    "wdr_dbg_cross_kv": (C.c_int, [vp, P(f32)]),
    "wdr_dbg_step": (C.c_int, [vp, P(i32), sz, P(f32)]),
    "wdr_dbg_logits": (C.c_int, [vp, P(f32), i32, P(i32), P(f32), f32, i32, P(i32), P(f32)]),
    "wdr_dbg_capture": (C.c_int, [vp, P(i32), sz, P(f32)]),
    "wdr_dbg_dtw": (C.c_int, [P(f32), i32, i32, i32, i32, i32, P(f32), P(i32), P(i32)]),
    "wdr_dbg_discrete": (C.c_int, [P(f32), sz, C.c_uint32, i32, P(i32)]),
    "wdr_dbg_dtw_dp": (C.c_int, [P(f32), i32, i32, i32, P(i32), P(i32)]),
    "wdr_dbg_proj": (C.c_int, [P(C.c_uint16), P(C.c_uint16), P(f32), i32, i32, i32, i32, P(f32)]),
    "wdr_dbg_proj_ln": (C.c_int, [P(f32), P(f32), P(f32), P(C.c_uint16), P(f32), i32, i32, i32, i32, i32, P(f32)]),
    "wdr_dbg_proj_fp8": (C.c_int, [P(C.c_uint16), P(C.c_uint16), P(f32), i32, i32, i32, i32, P(f32), P(C.c_uint8),
                                   P(C.c_uint8), P(C.c_uint8), P(C.c_uint8)]),
    "wdr_dbg_attn": (C.c_int, [P(C.c_uint16), P(C.c_uint16), P(C.c_uint16), i32, i32, i32, i32, P(f32)]),
    "wdr_dbg_xattn": (C.c_int, [P(C.c_uint16), P(C.c_uint16), P(i32), P(i32), i32, i32, i32, i32, P(f32)]),
}

_lib = None


class WdrError(RuntimeError):
    pass


def header_symbols():
    """Function names declared in include/wdr.h."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(wdr_[a-z0-9_]+)\s*\(", txt)))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise WdrError("libwdr.so not built at %s (run __graft_entry__.build())" % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    # release every handle still alive (contexts' worker threads, streams, device memory) before
    # the interpreter and the HIP runtime tear down; later frees of those handles are no-ops
    atexit.register(lib.wdr_shutdown)
    return lib


def check(rc: int):
    if rc != 0:
        raise WdrError(load().wdr_last_error().decode("utf-8", "replace"))
