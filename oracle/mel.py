"""Log-mel spectrogram, mel filterbank and signal energy (oracle side).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates whisper.cpp's `log_mel_spectrogram` + worker (reached from
`state.full`, src/transcribe.rs:389):
reflect-pad 200 samples at the start, zero-pad 30 s + 200 at the end,
periodic Hann(400), hop 160, |X|^2 over 201 bins, mel = filters . P,
log10(max(., 1e-10)), global clamp at (max - 8), then (x + 4) / 4.
Frames starting past the real samples evaluate to log10(1e-10) = -10.

`signal_energy` restates whisper.cpp `get_signal_energy(samples, n, 32)`
(token_timestamps=true, src/transcribe.rs:45; a3): f32 running sum of |x| over
[i-32, i+32] in index order, divided by 65.

`mel_filters` restates librosa.filters.mel(sr=16000, n_fft=400, norm='slaney')
(the filters whisper's ggml files embed); pinned against transformers'
`mel_filter_bank` in tests/golden.
"""
from __future__ import annotations

import numpy as np

SAMPLE_RATE = 16000
N_FFT = 400
HOP = 160
CHUNK_SAMPLES = 30 * SAMPLE_RATE


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filters(n_mels: int) -> np.ndarray:
    """[n_mels][201] float32 slaney filterbank (fmin 0, fmax 8000)."""
    n_bins = 1 + N_FFT // 2
    fftfreqs = np.linspace(0, SAMPLE_RATE / 2, n_bins)
    mel_pts = np.linspace(_hz_to_mel(0.0), _hz_to_mel(8000.0), n_mels + 2)
    mel_f = _mel_to_hz(mel_pts)
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, n_bins), np.float64)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    w *= enorm[:, None]
    return w.astype(np.float32)


def hann_periodic() -> np.ndarray:
    i = np.arange(N_FFT, dtype=np.float64)
    return (0.5 * (1.0 - np.cos(2.0 * np.pi * i / N_FFT))).astype(np.float32)


def mel_lengths(n: int):
    """(n_len, n_len_org) exactly as whisper.cpp computes them (C integer division)."""
    padded = n + CHUNK_SAMPLES + 2 * (N_FFT // 2)
    n_len = (padded - N_FFT) // HOP
    num = n + N_FFT // 2 - N_FFT
    n_len_org = 1 + int(num / HOP)   # C truncation toward zero
    return n_len, n_len_org


def log_mel(samples: np.ndarray, n_mels: int, filters: np.ndarray | None = None) -> np.ndarray:
    """[n_mels][n_len] float32 normalised log-mel of one `state.full` call."""
    x = np.asarray(samples, np.float32)
    n = x.shape[0]
    if filters is None:
        filters = mel_filters(n_mels)
    half = N_FFT // 2
    padded = np.zeros(n + CHUNK_SAMPLES + 2 * half, np.float32)
    padded[half:half + n] = x
    # std::reverse_copy(samples + 1, samples + 1 + 200, padded.begin())
    src = np.zeros(half, np.float32)
    m = max(0, min(half, n - 1))
    src[:m] = x[1:1 + m]
    padded[:half] = src[::-1]
    n_len, _ = mel_lengths(n)
    n_eff = n + half                      # worker's n_samples argument
    n_fft_frames = min(n_eff // HOP + 1, n_len)
    hann = hann_periodic()
    out = np.full((n_mels, n_len), -10.0, np.float64)
    if n_fft_frames > 0:
        idx = np.arange(n_fft_frames)[:, None] * HOP + np.arange(N_FFT)[None, :]
        frames = padded[idx]
        # samples at offset >= n_eff are zero already (padded region)
        frames = frames * hann[None, :]
        spec = np.fft.rfft(frames.astype(np.float64), axis=1)
        power = (spec.real ** 2 + spec.imag ** 2).astype(np.float32).astype(np.float64)
        mel = power @ filters.astype(np.float64).T        # [frames][n_mels], summed in double
        out[:, :n_fft_frames] = np.log10(np.maximum(mel, 1e-10)).T
    mmax = out.max() - 8.0
    out = np.maximum(out, mmax)
    out = (out + 4.0) / 4.0
    return out.astype(np.float32)


def signal_energy(samples: np.ndarray, hw: int = 32) -> np.ndarray:
    x = np.abs(np.asarray(samples, np.float32))
    n = x.shape[0]
    out = np.zeros(n, np.float32)
    # f32 accumulation in index order (bit-exact with the C loop)
    acc = np.zeros(n, np.float32)
    for j in range(-hw, hw + 1):
        lo, hi = max(0, -j), min(n, n - j)
        if hi <= lo:
            continue
        acc[lo:hi] = acc[lo:hi] + x[lo + j:hi + j]
    out[:] = acc / np.float32(2 * hw + 1)
    return out


def pcm_i16_to_f32(s: np.ndarray) -> np.ndarray:
    """whisper_rs::convert_integer_to_float_audio: x / 32768 (src/vad.rs:11-12, src/transcribe.rs:380-381)."""
    return (np.asarray(s, np.int16).astype(np.float32) / np.float32(32768.0)).astype(np.float32)
