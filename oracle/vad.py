"""Silero VAD v5.1.2 as whisper.cpp runs it.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the CPU restatement the HIP VAD
(csrc/kernels/vad.hip) is checked against.  Reference call site: src/vad.rs:15-31
(`WhisperVadContext::new`, `WhisperVadParams` with min_silence 100 ms, then
`segments_from_samples`); the merge that follows is oracle/pipeline.py:vad_merge
(src/vad.rs:33-84).

whisper.cpp (inside whisper-rs-sys, pinned whisper-rs 0.15.0 @ 0c509ec9) is not in the
container, so this restates its published algorithm:

  per 512-sample chunk (the last one zero-filled; one probability per chunk):
    reflect-pad 64 | 64  -> 640 samples
    STFT as conv1d: basis [258][256] (129 real rows, 129 imaginary rows), hop 128 -> 4 frames
    magnitude sqrt(re^2 + im^2)                                   -> [129][4]
    conv k3 s1 p1 129->128, ReLU; k3 s2 p1 128->64, ReLU; k3 s2 p1 64->64, ReLU;
    k3 s1 p1 64->128, ReLU                                          -> [128][1]
    LSTMCell(128): gates = W_ih x + b_ih + W_hh h + b_hh (i, f, g, o), state carried
      across every chunk of the call, zero at the start
    ReLU(h) -> conv k1 128->1 + b -> sigmoid                        -> p
  segments_from_probs: whisper.cpp's port of silero's get_speech_timestamps.

Numerics follow ggml: conv1d is im2col in f16 + mul_mat, so every conv / mul_mat input is
rounded to f16 against f16 weights, with f32 accumulation; elementwise ops are f32.

PARITY: unpinned against whisper.cpp itself (no executable reference or model file in the
container).  The details that are restated from memory of the published
code and flagged: reflect padding inside the STFT layer (no cross-chunk sample context),
zero fill of the last partial chunk, and f16 LSTM weights.

Synthetic weights (no model file offline): the STFT basis is the real one (Hann-windowed
DFT, as silero's forward_basis_buffer); every other tensor comes from the seeded generator
of oracle/weights.py under whisper.cpp-style tensor names.
"""
from __future__ import annotations

import math

import numpy as np

from .weights import synth_f16, synth_f32

N_WINDOW = 512
N_PAD = 64
N_FFT = 256
HOP = 128
N_BINS = 129
HID = 128

# (name, out, in, k, stride) of the four encoder convolutions
CONVS = [("_model.encoder.0.reparam_conv", 128, 129, 3, 1),
         ("_model.encoder.1.reparam_conv", 64, 128, 3, 2),
         ("_model.encoder.2.reparam_conv", 64, 64, 3, 2),
         ("_model.encoder.3.reparam_conv", 128, 64, 3, 1)]


def stft_basis() -> np.ndarray:
    """[258][256] f16: rows 0..128 = hann * cos(2 pi k t / 256), rows 129..257 = -hann * sin."""
    t = np.arange(N_FFT, dtype=np.float64)
    k = np.arange(N_BINS, dtype=np.float64)[:, None]
    hann = 0.5 - 0.5 * np.cos(2.0 * math.pi * t / N_FFT)          # periodic
    ang = 2.0 * math.pi * k * t / N_FFT
    b = np.concatenate([np.cos(ang) * hann, -np.sin(ang) * hann], 0)
    return b.astype(np.float16)


def vad_weights() -> dict:
    W = {"stft": stft_basis()}
    for name, o, i, k, _ in CONVS:
        W[name + ".weight"] = synth_f16(name + ".weight", (o, i, k), std=1.0 / math.sqrt(i * k))
        W[name + ".bias"] = synth_f32(name + ".bias", (o,), std=0.02)
    W["_model.decoder.rnn.weight_ih"] = synth_f16("_model.decoder.rnn.weight_ih", (4 * HID, HID), std=1.0 / math.sqrt(HID))
    W["_model.decoder.rnn.weight_hh"] = synth_f16("_model.decoder.rnn.weight_hh", (4 * HID, HID), std=1.0 / math.sqrt(HID))
    W["_model.decoder.rnn.bias_ih"] = synth_f32("_model.decoder.rnn.bias_ih", (4 * HID,), std=0.05)
    W["_model.decoder.rnn.bias_hh"] = synth_f32("_model.decoder.rnn.bias_hh", (4 * HID,), std=0.05)
    W["_model.decoder.decoder.2.weight"] = synth_f16("_model.decoder.decoder.2.weight", (1, HID, 1), std=3.0)
    W["_model.decoder.decoder.2.bias"] = synth_f32("_model.decoder.decoder.2.bias", (1,), std=0.02)
    return W


def _f16(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def _conv1d(x, w, b, stride):
    """x [B][C][T] f32, w [O][C][3] f16, pad 1 -> [B][O][T'] f32 (ggml_conv_1d: f16 im2col)."""
    B, C, T = x.shape
    xp = np.zeros((B, C, T + 2), np.float32)
    xp[:, :, 1:T + 1] = _f16(x)
    To = (T + 2 - 3) // stride + 1
    cols = np.stack([xp[:, :, s * stride:s * stride + 3] for s in range(To)], 1)   # [B][To][C][3]
    y = cols.reshape(B, To, C * 3).astype(np.float32) @ w.astype(np.float32).reshape(w.shape[0], -1).T
    return (y + b[None, None, :]).transpose(0, 2, 1).astype(np.float32)


def chunk_frames(x: np.ndarray) -> np.ndarray:
    """[n_chunks][640] padded chunk samples (f32)."""
    n = x.shape[0]
    nc = (n + N_WINDOW - 1) // N_WINDOW
    buf = np.zeros(nc * N_WINDOW, np.float32)
    buf[:n] = x
    c = buf.reshape(nc, N_WINDOW)
    left = c[:, 1:N_PAD + 1][:, ::-1]
    right = c[:, N_WINDOW - N_PAD - 1:N_WINDOW - 1][:, ::-1]
    return np.concatenate([left, c, right], 1)


def front(x: np.ndarray, W: dict) -> np.ndarray:
    """Everything before the recurrence, batched over chunks: [n_chunks][128] conv output."""
    fr = _f16(chunk_frames(x))                                          # [nc][640]
    nc = fr.shape[0]
    segs = np.stack([fr[:, HOP * f:HOP * f + N_FFT] for f in range(4)], 1)   # [nc][4][256]
    st = segs @ W["stft"].astype(np.float32).T                          # [nc][4][258]
    mag = np.sqrt(st[..., :N_BINS] ** 2 + st[..., N_BINS:] ** 2).astype(np.float32)
    h = mag.transpose(0, 2, 1)                                          # [nc][129][4]
    for name, _, _, _, stride in CONVS:
        h = np.maximum(_conv1d(h, W[name + ".weight"], W[name + ".bias"], stride), 0.0)
    assert h.shape[2] == 1
    return h[:, :, 0]


def probs(x: np.ndarray, W: dict) -> np.ndarray:
    """f32 [n_chunks] speech probabilities (whisper_vad_detect_speech)."""
    feat = front(np.asarray(x, np.float32), W)
    wih = W["_model.decoder.rnn.weight_ih"].astype(np.float32)
    whh = W["_model.decoder.rnn.weight_hh"].astype(np.float32)
    xg = (_f16(feat) @ wih.T + W["_model.decoder.rnn.bias_ih"]).astype(np.float32)
    wo = W["_model.decoder.decoder.2.weight"].astype(np.float32).reshape(HID)
    bo = np.float32(W["_model.decoder.decoder.2.bias"][0])
    h = np.zeros(HID, np.float32)
    c = np.zeros(HID, np.float32)
    out = np.zeros(feat.shape[0], np.float32)
    sig = lambda v: (1.0 / (1.0 + np.exp(-v))).astype(np.float32)
    for t in range(feat.shape[0]):
        g = xg[t] + (whh @ _f16(h) + W["_model.decoder.rnn.bias_hh"]).astype(np.float32)
        i, f, gg, o = sig(g[:HID]), sig(g[HID:2 * HID]), np.tanh(g[2 * HID:3 * HID]), sig(g[3 * HID:])
        c = (f * c + i * gg).astype(np.float32)
        h = (o * np.tanh(c)).astype(np.float32)
        out[t] = sig(np.float32(_f16(np.maximum(h, 0.0)) @ wo) + bo)
    return out


def segments_from_probs(p, threshold=0.5, min_speech_ms=250, min_silence_ms=100, max_speech_s=3.4028235e38,
                        speech_pad_ms=30):
    """whisper.cpp whisper_vad_segments_from_probs -> list of (start_cs, end_cs) f32 values.
    Defaults = whisper.cpp defaults with the reference's min_silence 100 ms (src/vad.rs:22)."""
    SR, NW = 16000, N_WINDOW
    n = len(p)
    min_sil = SR * min_silence_ms // 1000
    audio_len = n * NW
    min_speech = SR * min_speech_ms // 1000
    pad = SR * speech_pad_ms // 1000
    if max_speech_s > 100000.0:
        max_speech = (2 ** 31 - 1) // 2
    else:
        tmp = int(SR * int(max_speech_s)) - NW - 2 * pad
        max_speech = (2 ** 31 - 1) // 2 if (tmp > 2 ** 31 - 1 or tmp < 0) else tmp
    min_sil_at_max = SR * 98 // 1000
    neg = max(np.float32(threshold) - np.float32(0.15), np.float32(0.01))
    thr = np.float32(threshold)
    sp = []
    in_speech = False
    temp_end = prev_end = next_start = cur_start = 0
    has_cur = False
    for i in range(n):
        pr = np.float32(p[i])
        cs = NW * i
        if pr >= thr and temp_end:
            temp_end = 0
            if next_start < prev_end:
                next_start = cs
        if pr >= thr and not in_speech:
            in_speech = True
            cur_start = cs
            has_cur = True
            continue
        if in_speech and cs - cur_start > max_speech:
            if prev_end:
                sp.append([cur_start, prev_end])
                has_cur = True
                if next_start < prev_end:
                    in_speech = False
                    has_cur = False
                else:
                    cur_start = next_start
                prev_end = next_start = temp_end = 0
            else:
                sp.append([cur_start, cs])
                prev_end = next_start = temp_end = 0
                in_speech = False
                has_cur = False
                continue
        if pr < neg and in_speech:
            if not temp_end:
                temp_end = cs
            if cs - temp_end > min_sil_at_max:
                prev_end = temp_end
            if cs - temp_end < min_sil:
                continue
            if temp_end - cur_start > min_speech:
                sp.append([cur_start, temp_end])
            prev_end = next_start = temp_end = 0
            in_speech = False
            has_cur = False
            continue
    if has_cur and audio_len - cur_start > min_speech:
        sp.append([cur_start, audio_len])
    i = 0
    while i < len(sp) - 1:                         # merge gaps < 200 ms
        if sp[i + 1][0] - sp[i][1] < int(SR * 0.2):
            sp[i][1] = sp[i + 1][1]
            del sp[i + 1]
            continue
        i += 1
    sp = [s for s in sp if s[1] - s[0] >= min_speech]
    out = []
    for i in range(len(sp)):
        if i == 0:
            sp[i][0] = sp[i][0] - pad if sp[i][0] > pad else 0
        if i < len(sp) - 1:
            sil = sp[i + 1][0] - sp[i][1]
            if sil < 2 * pad:
                sp[i][1] += sil // 2
                sp[i + 1][0] = sp[i + 1][0] - sil // 2 if sp[i + 1][0] > sil // 2 else 0
            else:
                sp[i][1] = sp[i][1] + pad if sp[i][1] + pad < audio_len else audio_len
                sp[i + 1][0] = sp[i + 1][0] - pad if sp[i + 1][0] > pad else 0
        else:
            sp[i][1] = sp[i][1] + pad if sp[i][1] + pad < audio_len else audio_len
        out.append((float(np.float32(sp[i][0]) / np.float32(SR) * np.float32(100.0)),
                    float(np.float32(sp[i][1]) / np.float32(SR) * np.float32(100.0))))
    return out


def get_segments(int_samples: np.ndarray, W: dict | None = None):
    """src/vad.rs:6-85: (mask seconds, merged SpeechSegments)."""
    from .pipeline import vad_merge
    W = W if W is not None else vad_weights()
    x = np.asarray(int_samples, np.int16).astype(np.float32) / np.float32(32768.0)
    return vad_merge(segments_from_probs(probs(x, W)), np.asarray(int_samples, np.int16))
