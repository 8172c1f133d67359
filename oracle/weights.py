"""Whisper hyper-parameters and the synthetic, seeded weight generator (oracle side).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

There are no ggml checkpoints in this container, so both the
product (libwdr, csrc/whisper_model.cpp) and this oracle materialise the same
weights from a counter-based hash:

    seed   = FNV-1a-64(tensor name)
    h      = splitmix64(seed + i)            (i = flat element index, uint64)
    v      = float32(h >> 40) * 2**-23 - 1   (exact in f32, uniform [-1, 1))
    w      = float16(v * float32(std * sqrt(3)))

so both sides get bit-identical f16 weights.  Tensor names follow whisper.cpp's
ggml naming (model file layout: SURVEY.md §8(f) row 2).  2-D matrices are f16
(as in ggml files); biases, LayerNorm parameters and positional embeddings are
f32.  LayerNorm gamma = 1, beta = 0.
"""
from __future__ import annotations

import dataclasses
import math
import os

import numpy as np

M64 = (1 << 64) - 1


@dataclasses.dataclass(frozen=True)
class HParams:
    """ggml header hparams (SURVEY.md §8(a) table 'Model hparams')."""
    n_vocab: int = 51864
    n_audio_ctx: int = 1500
    n_audio_state: int = 512
    n_audio_head: int = 8
    n_audio_layer: int = 6
    n_text_ctx: int = 448
    n_text_state: int = 512
    n_text_head: int = 8
    n_text_layer: int = 6
    n_mels: int = 80

    @property
    def multilingual(self) -> bool:       # whisper.cpp whisper_is_multilingual: n_vocab >= 51865
        return self.n_vocab >= 51865

    @property
    def num_languages(self) -> int:       # large-v3 adds 'yue': n_vocab 51866
        return self.n_vocab - 51765 - (1 if self.multilingual else 0)


def hparams_for(name: str) -> HParams:
    """Named configs.  'base.en' and 'large-v3' are the BASELINE.json models;
    'tiny-test*' are reduced configs (d_head = 64 like every Whisper size) used by the
    parity tests so the numpy oracle finishes in seconds."""
    if name == "base.en":
        return HParams()
    if name == "large-v3":
        return HParams(n_vocab=51866, n_audio_state=1280, n_audio_head=20, n_audio_layer=32,
                       n_text_state=1280, n_text_head=20, n_text_layer=32, n_mels=128)
    if name == "tiny.en":
        return HParams(n_audio_state=384, n_audio_head=6, n_audio_layer=4,
                       n_text_state=384, n_text_head=6, n_text_layer=4)
    if name == "tiny-test":          # english-only token layout
        return HParams(n_audio_state=128, n_audio_head=2, n_audio_layer=2,
                       n_text_state=128, n_text_head=2, n_text_layer=2)
    if name == "tiny-test-ml":       # large-v3 token layout, 128 mels
        return HParams(n_vocab=51866, n_audio_state=128, n_audio_head=2, n_audio_layer=2,
                       n_text_state=128, n_text_head=2, n_text_layer=2, n_mels=128)
    raise KeyError(name)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & M64
    return h


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


_CHUNK = 1 << 18
_POOL = None


def _pool():
    """Threads for large tensors (numpy ufuncs release the GIL): BASELINE-size models
    (large-v3, 1.55 B parameters) are generated in seconds instead of minutes."""
    global _POOL
    if _POOL is None:
        import concurrent.futures
        _POOL = concurrent.futures.ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 1)))
    return _POOL


def _fill(seed: int, lo: int, hi: int, scale: np.float32, out: np.ndarray, round16: bool):
    with np.errstate(over="ignore"):
        idx = np.arange(lo, hi, dtype=np.uint64) + np.uint64(seed)
    h = splitmix64(idx)
    v = ((h >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -23) - np.float32(1.0)) * scale
    out[lo:hi] = v.astype(np.float16) if round16 else v


def _synth(name: str, n: int, std: float, dtype, round16: bool = False) -> np.ndarray:
    """dtype f16: the f16 tensor; f32 with round16: its values widened back to f32."""
    seed = fnv1a64(name)
    scale = np.float32(std * math.sqrt(3.0))
    out = np.empty(n, dtype)
    round16 = round16 or dtype == np.float16
    if n <= _CHUNK:
        _fill(seed, 0, n, scale, out, round16)
        return out
    futs = [_pool().submit(_fill, seed, lo, min(n, lo + _CHUNK), scale, out, round16) for lo in range(0, n, _CHUNK)]
    for f in futs:
        f.result()
    return out


def synth_uniform(name: str, n: int, std: float) -> np.ndarray:
    """f32 values (before the f16 cast) of a synthetic tensor with `n` elements."""
    return _synth(name, n, std, np.float32)


def synth_f16(name: str, shape, std: float = 0.02) -> np.ndarray:
    n = int(np.prod(shape))
    return _synth(name, n, std, np.float16).reshape(shape)


def synth_f32(name: str, shape, std: float = 0.02) -> np.ndarray:
    n = int(np.prod(shape))
    return synth_uniform(name, n, std).reshape(shape)


def tensor_list(hp: HParams):
    """(name, shape, kind) in whisper.cpp ggml naming; kind in {'w16','b32','ln_g','ln_b','p32'}."""
    d, dt = hp.n_audio_state, hp.n_text_state
    out = [
        ("encoder.conv1.weight", (d, hp.n_mels, 3), "w16"),
        ("encoder.conv1.bias", (d,), "b32"),
        ("encoder.conv2.weight", (d, d, 3), "w16"),
        ("encoder.conv2.bias", (d,), "b32"),
        ("encoder.positional_embedding", (hp.n_audio_ctx, d), "p32"),
    ]
    for i in range(hp.n_audio_layer):
        p = f"encoder.blocks.{i}."
        out += [
            (p + "attn_ln.weight", (d,), "ln_g"), (p + "attn_ln.bias", (d,), "ln_b"),
            (p + "attn.query.weight", (d, d), "w16"), (p + "attn.query.bias", (d,), "b32"),
            (p + "attn.key.weight", (d, d), "w16"),
            (p + "attn.value.weight", (d, d), "w16"), (p + "attn.value.bias", (d,), "b32"),
            (p + "attn.out.weight", (d, d), "w16"), (p + "attn.out.bias", (d,), "b32"),
            (p + "mlp_ln.weight", (d,), "ln_g"), (p + "mlp_ln.bias", (d,), "ln_b"),
            (p + "mlp.0.weight", (4 * d, d), "w16"), (p + "mlp.0.bias", (4 * d,), "b32"),
            (p + "mlp.2.weight", (d, 4 * d), "w16"), (p + "mlp.2.bias", (d,), "b32"),
        ]
    out += [("encoder.ln_post.weight", (d,), "ln_g"), ("encoder.ln_post.bias", (d,), "ln_b")]
    out += [
        ("decoder.token_embedding.weight", (hp.n_vocab, dt), "w16"),
        ("decoder.positional_embedding", (hp.n_text_ctx, dt), "p32"),
    ]
    for i in range(hp.n_text_layer):
        p = f"decoder.blocks.{i}."
        for a in ("attn", "cross_attn"):
            out += [
                (p + a + "_ln.weight", (dt,), "ln_g"), (p + a + "_ln.bias", (dt,), "ln_b"),
                (p + a + ".query.weight", (dt, dt), "w16"), (p + a + ".query.bias", (dt,), "b32"),
                (p + a + ".key.weight", (dt, dt), "w16"),
                (p + a + ".value.weight", (dt, dt), "w16"), (p + a + ".value.bias", (dt,), "b32"),
                (p + a + ".out.weight", (dt, dt), "w16"), (p + a + ".out.bias", (dt,), "b32"),
            ]
        out += [
            (p + "mlp_ln.weight", (dt,), "ln_g"), (p + "mlp_ln.bias", (dt,), "ln_b"),
            (p + "mlp.0.weight", (4 * dt, dt), "w16"), (p + "mlp.0.bias", (4 * dt,), "b32"),
            (p + "mlp.2.weight", (dt, 4 * dt), "w16"), (p + "mlp.2.bias", (dt,), "b32"),
        ]
    out += [("decoder.ln.weight", (dt,), "ln_g"), ("decoder.ln.bias", (dt,), "ln_b")]
    return out


def synth_weights(hp: HParams, std: float = 0.02, emb_std: float | None = None) -> dict:
    """All tensors as float32 numpy arrays holding the exact values the GPU sees
    (f16 matrices already rounded).  `emb_std` overrides the token-embedding std."""
    W = {}
    for name, shape, kind in tensor_list(hp):
        if kind == "w16":
            s = emb_std if (emb_std is not None and name == "decoder.token_embedding.weight") else std
            W[name] = _synth(name, int(np.prod(shape)), s, np.float32, round16=True).reshape(shape)
        elif kind in ("b32", "p32"):
            W[name] = synth_f32(name, shape, std)
        elif kind == "ln_g":
            W[name] = np.ones(shape, np.float32)
        else:
            W[name] = np.zeros(shape, np.float32)
    return W
