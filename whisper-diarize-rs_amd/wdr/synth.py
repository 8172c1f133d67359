"""Synthetic speech-like 16 kHz mono audio (SURVEY.md §8(d) 'Synthetic inputs').

Talk spurts U[1.5, 8.0] s separated by pauses U[0.3, 1.5] s; spurts are
syllables of 120-250 ms (raised-cosine envelope) built from harmonics of F0
(<= 4 kHz) shaped by three per-syllable formants; speakers F0 in
{110, 140, 190, 230} Hz +-5 %, round-robin per spurt; -12 dBFS RMS in spurts,
-60 dBFS white noise elsewhere.  Deterministic for a given seed.

Returns the int16 samples and the ground-truth spurt table
[(start_s, end_s, speaker_index)] which the synthetic workload pin uses as the
segment list.
"""
from __future__ import annotations

import numpy as np

SR = 16000
F0S = (110.0, 140.0, 190.0, 230.0)


def synth_speech(duration_s: float, seed: int = 0, n_speakers: int = 1):
    rng = np.random.default_rng(seed)
    n = int(round(duration_s * SR))
    noise_rms = 10 ** (-60 / 20)
    out = (rng.standard_normal(n) * noise_rms).astype(np.float32)
    speech_rms = 10 ** (-12 / 20)
    spurts = []
    t = float(rng.uniform(0.3, 1.5))
    k = 0
    while True:
        dur = float(rng.uniform(1.5, 8.0))
        if t + dur > duration_s - 0.3:
            break
        spk = k % n_speakers
        f0_base = F0S[spk]
        s0 = int(round(t * SR))
        s1 = int(round((t + dur) * SR))
        pos = s0
        seg = np.zeros(s1 - s0, np.float32)
        while pos < s1:
            L = int(rng.uniform(0.120, 0.250) * SR)
            L = min(L, s1 - pos)
            if L < 32:
                break
            f0 = f0_base * float(rng.uniform(0.95, 1.05))
            F = (rng.uniform(300, 800), rng.uniform(900, 2300), rng.uniform(2500, 3000))
            tt = np.arange(L, dtype=np.float64) / SR
            nh = int(4000 // f0)
            h = np.arange(1, nh + 1, dtype=np.float64)
            fr = h * f0
            gain = np.zeros_like(fr)
            for fc, bw in zip(F, (80.0, 120.0, 160.0)):
                gain += 1.0 / (1.0 + ((fr - fc) / bw) ** 2)
            gain /= np.sqrt(h)
            ph = rng.uniform(0, 2 * np.pi, nh)
            wave = (gain[None, :] * np.sin(2 * np.pi * fr[None, :] * tt[:, None] + ph[None, :])).sum(1)
            env = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(L) / max(L - 1, 1))
            env *= 0.75 + 0.25 * np.sin(2 * np.pi * 4.0 * tt)
            syl = wave * env
            seg[pos - s0:pos - s0 + L] = syl.astype(np.float32)
            pos += L
        rms = float(np.sqrt(np.mean(seg.astype(np.float64) ** 2)) + 1e-12)
        out[s0:s1] += seg * np.float32(speech_rms / rms)
        spurts.append((s0 / SR, s1 / SR, spk))
        t += dur + float(rng.uniform(0.3, 1.5))
        k += 1
    pcm = np.clip(np.round(out * 32767.0), -32768, 32767).astype(np.int16)
    return pcm, spurts
