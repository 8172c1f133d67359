"""Whisper encoder / decoder forward in numpy (oracle side).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates the ggml graphs whisper.cpp builds inside `state.full`
(src/transcribe.rs:389), including
the ggml rounding points, so the numerics match what the reference computes:

* mul_mat with f16 weights converts the f32 activation to f16 first
  (`f16in=True` rounds activations to f16, accumulation f32);
* conv1d goes through an f16 im2col;
* Q, K, V (self), cross K/V and the KV cache are stored f16; softmax in f32,
  the probabilities enter P.V as f16;
* GELU is the tanh approximation; LayerNorm eps 1e-5 (biased variance);
* cross-attention keys/queries scaled by d_head^-1/2 overall.

With `f16in=False` the graph is plain f32 and is pinned against
transformers' WhisperModel (activation 'gelu_new') in tests/golden.
"""
from __future__ import annotations

import numpy as np

from .weights import HParams

EPS = 1e-5


def f16(x):
    return x.astype(np.float16).astype(np.float32)


class Rounding:
    def __init__(self, f16in: bool = True):
        self.on = f16in

    def __call__(self, x):
        return f16(x) if self.on else x.astype(np.float32)


def layer_norm(x, g, b, eps=EPS):
    x = x.astype(np.float32)
    mu = x.mean(-1, keepdims=True, dtype=np.float64)
    var = ((x - mu) ** 2).mean(-1, keepdims=True, dtype=np.float64)
    return ((x - mu) / np.sqrt(var + eps) * g + b).astype(np.float32)


def gelu_tanh(x):
    x = x.astype(np.float32)
    return (0.5 * x * (1.0 + np.tanh(np.float32(0.7978845608028654) * (x + np.float32(0.044715) * x * x * x)))).astype(np.float32)


def gelu_erf(x):
    from scipy.special import erf
    x = x.astype(np.float64)
    return (0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))).astype(np.float32)


def linear(x, w, b, R):
    y = R(x) @ w.T
    if b is not None:
        y = y + b
    return y.astype(np.float32)


def softmax(s, axis=-1):
    m = s.max(axis=axis, keepdims=True)
    e = np.exp(s - m)
    return (e / e.sum(axis=axis, keepdims=True)).astype(np.float32)


def attention(q, k, v, n_head, R, mask=None, want_probs=False, kv_rounded=False):
    """q [Tq][d], k/v [Tk][d] (already projected).  Returns [Tq][d] (and probs [H][Tq][Tk]).
    kv_rounded: k and v already hold R-rounded values (caches), R is idempotent -- skipped."""
    Tq, d = q.shape
    dh = d // n_head
    qh = R(q).reshape(Tq, n_head, dh).transpose(1, 0, 2)
    kh = (k if kv_rounded else R(k)).reshape(-1, n_head, dh).transpose(1, 0, 2)
    vh = (v if kv_rounded else R(v)).reshape(-1, n_head, dh).transpose(1, 0, 2)
    s = (qh @ kh.transpose(0, 2, 1)) * np.float32(dh ** -0.5)
    if mask is not None:
        s = s + mask
    p = softmax(s)
    o = (R(p) @ vh).transpose(1, 0, 2).reshape(Tq, d)
    return (o, p) if want_probs else o


class Whisper:
    def __init__(self, hp: HParams, W: dict, f16in: bool = True, conv_act=None):
        self.hp, self.W, self.R = hp, W, Rounding(f16in)
        # whisper.cpp applies ggml_gelu (tanh form) after both convs; transformers uses the
        # exact erf GELU there — selectable only so the f32 graph can be pinned against it.
        self.conv_act = conv_act or gelu_tanh

    # ---------------- encoder (a5, a6) ----------------
    def conv1d(self, x, w, b, stride):
        """x [Cin][T] -> [Tout][Cout]; k=3, pad=1 (ggml_conv_1d_ph), f16 im2col."""
        Cin, T = x.shape
        xp = np.zeros((Cin, T + 2), np.float32)
        xp[:, 1:T + 1] = self.R(x)
        Tout = (T + 2 - 3) // stride + 1
        cols = np.stack([xp[:, k:k + stride * (Tout - 1) + 1:stride] for k in range(3)], axis=-1)  # [Cin][Tout][3]
        cols = cols.transpose(1, 0, 2).reshape(Tout, Cin * 3)
        y = cols @ w.reshape(w.shape[0], -1).T + b
        return y.astype(np.float32)

    def encode(self, mel_window):
        """mel_window [n_mels][3000] -> encoder output [1500][d] (after ln_post)."""
        W, R, hp = self.W, self.R, self.hp
        x = self.conv_act(self.conv1d(mel_window, W["encoder.conv1.weight"], W["encoder.conv1.bias"], 1))
        x = self.conv_act(self.conv1d(x.T, W["encoder.conv2.weight"], W["encoder.conv2.bias"], 2))
        x = (x + W["encoder.positional_embedding"][:x.shape[0]]).astype(np.float32)
        for i in range(hp.n_audio_layer):
            p = f"encoder.blocks.{i}."
            h = layer_norm(x, W[p + "attn_ln.weight"], W[p + "attn_ln.bias"])
            q = linear(h, W[p + "attn.query.weight"], W[p + "attn.query.bias"], R)
            k = linear(h, W[p + "attn.key.weight"], None, R)
            v = linear(h, W[p + "attn.value.weight"], W[p + "attn.value.bias"], R)
            a = attention(q, k, v, hp.n_audio_head, R)
            x = x + linear(a, W[p + "attn.out.weight"], W[p + "attn.out.bias"], R)
            h = layer_norm(x, W[p + "mlp_ln.weight"], W[p + "mlp_ln.bias"])
            h = gelu_tanh(linear(h, W[p + "mlp.0.weight"], W[p + "mlp.0.bias"], R))
            x = x + linear(h, W[p + "mlp.2.weight"], W[p + "mlp.2.bias"], R)
        return layer_norm(x, W["encoder.ln_post.weight"], W["encoder.ln_post.bias"])

    def cross_kv(self, enc):
        """a7: per decoder layer K = H.Wk (no bias), V = H.Wv + bv, stored f16."""
        W, R = self.W, self.R
        out = []
        for i in range(self.hp.n_text_layer):
            p = f"decoder.blocks.{i}.cross_attn."
            k = linear(enc, W[p + "key.weight"], None, R)
            v = linear(enc, W[p + "value.weight"], W[p + "value.bias"], R)
            out.append((R(k), R(v)))
        return out


class DecoderState:
    """Self-attention KV cache for ONE decoder sequence (f16-rounded values)."""

    def __init__(self, model: Whisper):
        self.m = model
        L = model.hp.n_text_layer
        self.k = [np.zeros((0, model.hp.n_text_state), np.float32) for _ in range(L)]
        self.v = [np.zeros((0, model.hp.n_text_state), np.float32) for _ in range(L)]

    def copy(self):
        s = DecoderState.__new__(DecoderState)
        s.m = self.m
        s.k = [a.copy() for a in self.k]
        s.v = [a.copy() for a in self.v]
        return s

    @property
    def n_past(self):
        return self.k[0].shape[0]

    def forward(self, tokens, cross, want_logits="last", aheads=None):
        """Run the decoder over `tokens` appended after the cached ones.
        Returns logits [n][n_vocab] ("last" -> [n_vocab] of the last token, None -> no logits)
        and, if `aheads` is a list of (layer, head), the cross-attention probabilities
        [len(aheads)][n][1500]."""
        m, W, R, hp = self.m, self.m.W, self.m.R, self.m.hp
        n = len(tokens)
        pos0 = self.n_past
        x = (W["decoder.token_embedding.weight"][np.asarray(tokens)]
             + W["decoder.positional_embedding"][pos0:pos0 + n]).astype(np.float32)
        captured = {}
        for i in range(hp.n_text_layer):
            p = f"decoder.blocks.{i}."
            h = layer_norm(x, W[p + "attn_ln.weight"], W[p + "attn_ln.bias"])
            q = linear(h, W[p + "attn.query.weight"], W[p + "attn.query.bias"], R)
            k = linear(h, W[p + "attn.key.weight"], None, R)
            v = linear(h, W[p + "attn.value.weight"], W[p + "attn.value.bias"], R)
            self.k[i] = np.concatenate([self.k[i], R(k)])
            self.v[i] = np.concatenate([self.v[i], R(v)])
            T = self.k[i].shape[0]
            mask = np.zeros((n, T), np.float32)
            for r in range(n):
                mask[r, pos0 + r + 1:] = -np.inf
            a = attention(q, self.k[i], self.v[i], hp.n_text_head, R, mask=mask[None], kv_rounded=True)
            x = x + linear(a, W[p + "attn.out.weight"], W[p + "attn.out.bias"], R)
            h = layer_norm(x, W[p + "cross_attn_ln.weight"], W[p + "cross_attn_ln.bias"])
            q = linear(h, W[p + "cross_attn.query.weight"], W[p + "cross_attn.query.bias"], R)
            ck, cv = cross[i]
            a, probs = attention(q, ck, cv, hp.n_text_head, R, want_probs=True, kv_rounded=True)
            if aheads:
                for (l, hh) in aheads:
                    if l == i:
                        captured[(l, hh)] = probs[hh]
            x = x + linear(a, W[p + "cross_attn.out.weight"], W[p + "cross_attn.out.bias"], R)
            h = layer_norm(x, W[p + "mlp_ln.weight"], W[p + "mlp_ln.bias"])
            h = gelu_tanh(linear(h, W[p + "mlp.0.weight"], W[p + "mlp.0.bias"], R))
            x = x + linear(h, W[p + "mlp.2.weight"], W[p + "mlp.2.bias"], R)
        logits = None
        if want_logits is not None:
            h = layer_norm(x, W["decoder.ln.weight"], W["decoder.ln.bias"])
            if want_logits == "last":
                h = h[-1:]
            logits = linear(h, W["decoder.token_embedding.weight"], None, R)
            if want_logits == "last":
                logits = logits[0]
        if aheads:
            return logits, np.stack([captured[a] for a in aheads])
        return logits
