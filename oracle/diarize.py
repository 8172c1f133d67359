"""Diarization path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the CPU restatement (numpy f32) the HIP
diarization kernels (csrc/kernels/diar.hip, csrc/diarize.cpp) are checked against.

Reference call sites: pyannote_rs::get_segments (src/engine.rs:117-122), EmbeddingExtractor
::compute + EmbeddingManager (src/transcribe.rs:339-345, 461-497).  pyannote-rs 0.3.1 @
546f35bc, ONNX Runtime, kaldi-native-fbank and the two ONNX models are network dependencies
absent from the container, so this restates their published algorithms:

  a16 segmentation-3.0 (PyanNet): per 10-s window of raw (unnormalised) int16-valued f32:
      InstanceNorm(1) -> SincNet [conv 80 x k251 s10 -> |.| -> maxpool 3 -> InstanceNorm ->
      LeakyReLU; conv 60 k5 -> maxpool 3 -> IN -> LReLU; conv 60 k5 -> maxpool 3 -> IN ->
      LReLU] (589 frames) -> 4-layer BiLSTM(128) -> Linear 256->128, LReLU -> Linear 128->128,
      LReLU -> Linear 128->7 -> log-softmax.  get_segments stitches frame argmax != 0 runs.
  a17 Kaldi fbank: 25 ms / 10 ms frames (snip edges), DC removal, pre-emphasis 0.97, Povey
      window, 512-point power spectrum, 80 triangular mel bins 20 Hz .. 8 kHz, log(max(e,
      FLT_EPSILON)); then the per-utterance mean is subtracted (knf-rs compute_fbank).
  a18 CAM++ (wespeaker CAMPPlus, 512-d): FCM 2-D front-end -> TDNN -> 3 CAM dense blocks
      (12/24/16 layers, growth 32, dilation 1/2/2) with transit layers -> BN-ReLU -> stats
      pooling (mean, unbiased std) -> dense 1024->512 + BN (no affine).
  a19 EmbeddingManager: cosine similarity; search_speaker (strictly greater than the
      threshold, else a new id while below max_speakers) / get_best_speaker_match.

Inference-mode BatchNorm is an affine map per channel (scale, shift) -- that is what the
ONNX graphs hold after export -- so the synthetic weights give each BN a seeded scale
(1 + u) and shift.

PARITY: unpinned (no executable reference, model or fixture for these rows in the
container); flagged details: the pyannote-rs iterator's early stop when a
window yields no segment (restated as published), knf input scale (x / 32768), the
Nyquist bin excluded from the mel banks (Kaldi).

Synthetic weights come from the seeded generator of oracle/weights.py (f32, uniform with
the given std) under ONNX-like parameter names.
"""
from __future__ import annotations

import math

import numpy as np

from .weights import synth_f32

# ------------------------------------------------------------------ common layers
LRELU = np.float32(0.01)


def _lrelu(x):
    return np.where(x >= 0, x, x * LRELU).astype(np.float32)


def _inorm(x, g, b, eps=1e-5):
    """InstanceNorm1d(affine) over time; x [C][T]."""
    m = x.mean(1, keepdims=True, dtype=np.float64)
    v = ((x - m) ** 2).mean(1, keepdims=True, dtype=np.float64)
    return (((x - m) / np.sqrt(v + eps)) * g[:, None] + b[:, None]).astype(np.float32)


def _conv1d(x, w, b=None, stride=1, pad=0, dil=1):
    """x [C][T] f32, w [O][C][k] -> [O][T']."""
    C, T = x.shape
    O, _, k = w.shape
    xp = np.pad(x, ((0, 0), (pad, pad)))
    To = (T + 2 * pad - dil * (k - 1) - 1) // stride + 1
    if To <= 0:
        return np.zeros((O, 0), np.float32)
    idx = np.arange(To)[:, None] * stride + np.arange(k)[None, :] * dil     # [To][k]
    cols = xp[:, idx]                                                        # [C][To][k]
    cols = cols.transpose(1, 0, 2).reshape(To, C * k)
    y = cols @ w.reshape(O, C * k).T
    if b is not None:
        y = y + b[None, :]
    return y.T.astype(np.float32)


def _maxpool3(x):
    C, T = x.shape
    To = T // 3
    return x[:, :To * 3].reshape(C, To, 3).max(2)


def _lstm_dir(x, wih, whh, bih, bhh, reverse):
    """x [T][I] -> [T][H] (torch gate order i, f, g, o; zero initial state)."""
    T = x.shape[0]
    H = whh.shape[1]
    xg = (x @ wih.T + bih).astype(np.float32)
    h = np.zeros(H, np.float32)
    c = np.zeros(H, np.float32)
    out = np.zeros((T, H), np.float32)
    sig = lambda v: (1.0 / (1.0 + np.exp(-v))).astype(np.float32)
    rng = range(T - 1, -1, -1) if reverse else range(T)
    for t in rng:
        g = xg[t] + (whh @ h + bhh)
        i, f, gg, o = sig(g[:H]), sig(g[H:2 * H]), np.tanh(g[2 * H:3 * H]), sig(g[3 * H:])
        c = (f * c + i * gg).astype(np.float32)
        h = (o * np.tanh(c)).astype(np.float32)
        out[t] = h
    return out


# ------------------------------------------------------------------ a16 segmentation-3.0
SEG_WIN = 160000
SEG_FRAMES = 589
FRAME_START = 721
FRAME_SIZE = 270
SEG_CLASS0_OFFSET = 0.86


def seg_weights() -> dict:
    W = {}
    f = lambda n, shape, std: W.__setitem__(n, synth_f32("seg." + n, shape, std))
    one = lambda n, c, std=0.1: W.__setitem__(n, (synth_f32("seg." + n, (c,), std) + np.float32(1.0)).astype(np.float32))
    one("wav_norm.weight", 1)
    f("wav_norm.bias", (1,), 0.1)
    f("sinc.weight", (80, 1, 251), 1.0 / math.sqrt(251))
    for i, c in enumerate((80, 60, 60)):
        one("norm%d.weight" % i, c)
        f("norm%d.bias" % i, (c,), 0.1)
    f("conv1.weight", (60, 80, 5), 1.0 / math.sqrt(400))
    f("conv1.bias", (60,), 0.05)
    f("conv2.weight", (60, 60, 5), 1.0 / math.sqrt(300))
    f("conv2.bias", (60,), 0.05)
    for l in range(4):
        I = 60 if l == 0 else 256
        for d in ("", "_reverse"):
            f("lstm.weight_ih_l%d%s" % (l, d), (512, I), 1.0 / math.sqrt(128))
            f("lstm.weight_hh_l%d%s" % (l, d), (512, 128), 1.0 / math.sqrt(128))
            f("lstm.bias_ih_l%d%s" % (l, d), (512,), 0.05)
            f("lstm.bias_hh_l%d%s" % (l, d), (512,), 0.05)
    f("linear0.weight", (128, 256), 1.0 / math.sqrt(256))
    f("linear0.bias", (128,), 0.05)
    f("linear1.weight", (128, 128), 1.0 / math.sqrt(128))
    f("linear1.bias", (128,), 0.05)
    f("classifier.weight", (7, 128), 8.0 / math.sqrt(128))
    f("classifier.bias", (7,), 0.05)
    # synthetic calibration: centre the class-0 ("no speaker") margin so that frames split
    # between silence and speech and get_segments sees runs of both
    W["classifier.bias"][0] += np.float32(SEG_CLASS0_OFFSET)
    return W


def seg_features(win: np.ndarray, W: dict) -> np.ndarray:
    """SincNet: [160000] f32 -> [60][589]."""
    x = _inorm(np.asarray(win, np.float32)[None, :], W["wav_norm.weight"], W["wav_norm.bias"])
    x = np.abs(_conv1d(x, W["sinc.weight"], None, stride=10))            # [80][15975]
    x = _lrelu(_inorm(_maxpool3(x), W["norm0.weight"], W["norm0.bias"]))
    x = _conv1d(x, W["conv1.weight"], W["conv1.bias"])
    x = _lrelu(_inorm(_maxpool3(x), W["norm1.weight"], W["norm1.bias"]))
    x = _conv1d(x, W["conv2.weight"], W["conv2.bias"])
    x = _lrelu(_inorm(_maxpool3(x), W["norm2.weight"], W["norm2.bias"]))
    return x


def seg_window(win: np.ndarray, W: dict) -> np.ndarray:
    """[160000] -> log-probabilities [589][7]."""
    h = seg_features(win, W).T                                            # [589][60]
    for l in range(4):
        outs = []
        for d, rev in (("", False), ("_reverse", True)):
            outs.append(_lstm_dir(h, W["lstm.weight_ih_l%d%s" % (l, d)], W["lstm.weight_hh_l%d%s" % (l, d)],
                                  W["lstm.bias_ih_l%d%s" % (l, d)], W["lstm.bias_hh_l%d%s" % (l, d)], rev))
        h = np.concatenate(outs, 1)
    h = _lrelu(h @ W["linear0.weight"].T + W["linear0.bias"])
    h = _lrelu(h @ W["linear1.weight"].T + W["linear1.bias"])
    z = (h @ W["classifier.weight"].T + W["classifier.bias"]).astype(np.float32)
    m = z.max(1, keepdims=True)
    return (z - m - np.log(np.exp(z - m).sum(1, keepdims=True))).astype(np.float32)


def last_argmax(row) -> int:
    """pyannote-rs find_max_index: Iterator::max_by keeps the LAST maximal element."""
    best, bi = None, 0
    for i, v in enumerate(row):
        if best is None or not (v < best):
            best, bi = v, i
    return bi


def get_segments_from_argmax(n_samples: int, frame_cls, early_stop: bool = True):
    """pyannote_rs::get_segments stitching over per-window frame classes [n_windows][589]
    -> [(start_s, end_s, start_idx, end_idx)] with indices into the padded buffer."""
    win = SEG_WIN
    padded = n_samples + (win - n_samples % win)
    offset = FRAME_START
    speaking = False
    start_offset = 0.0
    queue, out = [], []
    for w in range(padded // win):
        for k in range(SEG_FRAMES):
            if frame_cls[w][k] != 0:
                if not speaking:
                    start_offset = float(offset)
                    speaking = True
            elif speaking:
                start = start_offset / 16000.0
                end = offset / 16000.0
                si = int(min(start * 16000.0, float(padded - 1)))
                ei = int(min(end * 16000.0, float(padded)))
                speaking = False
                queue.append((start, end, si, ei))
            offset += FRAME_SIZE
        if queue:
            out.append(queue.pop(0))
        elif early_stop:
            return out
    return out + queue


def get_segments(samples_i16: np.ndarray, W: dict | None = None):
    W = W if W is not None else seg_weights()
    x = np.asarray(samples_i16, np.int16)
    n = x.size
    padded = np.zeros(n + (SEG_WIN - n % SEG_WIN), np.float32)
    padded[:n] = x
    cls = [[last_argmax(r) for r in seg_window(padded[s:s + SEG_WIN], W)] for s in range(0, padded.size, SEG_WIN)]
    return get_segments_from_argmax(n, cls)


# ------------------------------------------------------------------ a17 Kaldi fbank
def _mel(f):
    return 1127.0 * np.log(1.0 + f / 700.0)


def kaldi_mel_banks(num_bins=80, n_fft=512, sr=16000.0, low=20.0, high=0.0) -> np.ndarray:
    """[num_bins][n_fft/2] f32 (Kaldi MelBanks; the Nyquist bin is not covered)."""
    nyq = 0.5 * sr
    if high <= 0.0:
        high = nyq + high
    nfb = n_fft // 2
    bw = sr / n_fft
    ml, mh = _mel(low), _mel(high)
    delta = (mh - ml) / (num_bins + 1)
    out = np.zeros((num_bins, nfb), np.float32)
    for b in range(num_bins):
        left, center, right = ml + b * delta, ml + (b + 1) * delta, ml + (b + 2) * delta
        for i in range(nfb):
            m = _mel(bw * i)
            if left < m < right:
                out[b, i] = (m - left) / (center - left) if m <= center else (right - m) / (right - center)
    return out


def povey_window(n=400) -> np.ndarray:
    i = np.arange(n, dtype=np.float64)
    return np.power(0.5 - 0.5 * np.cos(2.0 * math.pi * i / (n - 1)), 0.85).astype(np.float32)


def fbank(samples_f32: np.ndarray) -> np.ndarray:
    """[T][80] log mel energies (before mean subtraction), snip_edges framing."""
    x = np.asarray(samples_f32, np.float32)
    n = x.size
    T = 0 if n < 400 else 1 + (n - 400) // 160
    if T == 0:
        return np.zeros((0, 80), np.float32)
    idx = np.arange(T)[:, None] * 160 + np.arange(400)[None, :]
    fr = x[idx].astype(np.float32)
    fr = fr - fr.mean(1, keepdims=True, dtype=np.float64).astype(np.float32)
    pe = fr.copy()
    pe[:, 1:] = fr[:, 1:] - np.float32(0.97) * fr[:, :-1]
    pe[:, 0] = fr[:, 0] - np.float32(0.97) * fr[:, 0]
    pe = pe * povey_window()[None, :]
    spec = np.fft.rfft(pe.astype(np.float64), n=512, axis=1)
    power = (spec.real ** 2 + spec.imag ** 2)[:, :256].astype(np.float32)
    e = power @ kaldi_mel_banks().T
    return np.log(np.maximum(e, np.float32(np.finfo(np.float32).eps))).astype(np.float32)


def compute_feats(samples_i16: np.ndarray) -> np.ndarray:
    """EmbeddingExtractor::compute's features: i16 / 32768 -> fbank -> minus the mean."""
    f = fbank(np.asarray(samples_i16, np.int16).astype(np.float32) / np.float32(32768.0))
    if f.shape[0] == 0:
        return f
    return (f - f.mean(0, keepdims=True, dtype=np.float64).astype(np.float32)).astype(np.float32)


# ------------------------------------------------------------------ a18 CAM++
CAM_BLOCKS = ((12, 3, 1), (24, 3, 2), (16, 3, 2))
GROWTH, BN_CH, INIT_CH = 32, 128, 128


def _bn(W, name, c):
    W[name + ".scale"] = (synth_f32("cam." + name + ".scale", (c,), 0.1) + np.float32(1.0)).astype(np.float32)
    W[name + ".shift"] = synth_f32("cam." + name + ".shift", (c,), 0.1)


def cam_weights() -> dict:
    W = {}
    f = lambda n, shape, std: W.__setitem__(n, synth_f32("cam." + n, shape, std))
    m = 32
    f("head.conv1", (m, 1, 3, 3), 1.0 / 3.0)
    _bn(W, "head.bn1", m)
    for L in (1, 2):
        for b in range(2):
            p = "head.layer%d.%d" % (L, b)
            f(p + ".conv1", (m, m, 3, 3), 1.0 / math.sqrt(9 * m))
            _bn(W, p + ".bn1", m)
            f(p + ".conv2", (m, m, 3, 3), 1.0 / math.sqrt(9 * m))
            _bn(W, p + ".bn2", m)
            if b == 0:
                f(p + ".shortcut", (m, m, 1, 1), 1.0 / math.sqrt(m))
                _bn(W, p + ".shortcut_bn", m)
    f("head.conv2", (m, m, 3, 3), 1.0 / math.sqrt(9 * m))
    _bn(W, "head.bn2", m)
    f("tdnn.linear", (INIT_CH, 320, 5), 1.0 / math.sqrt(320 * 5))
    _bn(W, "tdnn.bn", INIT_CH)
    ch = INIT_CH
    for bi, (nl, k, dil) in enumerate(CAM_BLOCKS):
        for li in range(nl):
            p = "block%d.%d" % (bi + 1, li)
            cin = ch + li * GROWTH
            _bn(W, p + ".bn1", cin)
            f(p + ".linear1", (BN_CH, cin, 1), 1.0 / math.sqrt(cin))
            _bn(W, p + ".bn2", BN_CH)
            f(p + ".local", (GROWTH, BN_CH, k), 1.0 / math.sqrt(BN_CH * k))
            f(p + ".cam1.weight", (BN_CH // 2, BN_CH, 1), 1.0 / math.sqrt(BN_CH))
            f(p + ".cam1.bias", (BN_CH // 2,), 0.05)
            f(p + ".cam2.weight", (GROWTH, BN_CH // 2, 1), 1.0 / math.sqrt(BN_CH // 2))
            f(p + ".cam2.bias", (GROWTH,), 0.05)
        ch = ch + nl * GROWTH
        _bn(W, "transit%d.bn" % (bi + 1), ch)
        f("transit%d.linear" % (bi + 1), (ch // 2, ch, 1), 1.0 / math.sqrt(ch))
        ch //= 2
    _bn(W, "out.bn", ch)
    f("dense.linear", (512, 2 * ch, 1), 1.0 / math.sqrt(2 * ch))
    _bn(W, "dense.bn", 512)
    return W


def cam_weights_conditioned(path: str) -> dict:
    """cam_weights() with a speaker-conditioned last layer (tests/golden/make_cam_conditioning.py:
    e = R P (dense.linear @ stats - mu), fitted on a calibration recording): dense.linear' =
    R P dense.linear, its BN scale 1 and shift -R P mu.  Test infrastructure: the diarized
    fixtures' embedding network, written for the GPU by tests/model_writers.py."""
    W = cam_weights()
    c = np.load(path)
    RP = c["R"].astype(np.float64) @ c["P"].astype(np.float64)                  # [512][512]
    dl = W["dense.linear"]
    W["dense.linear"] = (RP @ dl.reshape(512, -1).astype(np.float64)).astype(np.float32).reshape(dl.shape)
    W["dense.bn.scale"] = np.ones(512, np.float32)
    W["dense.bn.shift"] = (-(RP @ c["mu"].astype(np.float64))).astype(np.float32)
    return W


def _affine(x, W, name, axis=0):
    s, b = W[name + ".scale"], W[name + ".shift"]
    shape = [1] * x.ndim
    shape[axis] = -1
    return (x * s.reshape(shape) + b.reshape(shape)).astype(np.float32)


def _conv2d(x, w, stride_f=1):
    """x [C][F][T], w [O][C][3|1][3|1], pad (k-1)/2, stride (stride_f, 1) -> [O][F'][T]."""
    C, F, T = x.shape
    O, _, kf, kt = w.shape
    pf, pt = (kf - 1) // 2, (kt - 1) // 2
    xp = np.pad(x, ((0, 0), (pf, pf), (pt, pt)))
    Fo = (F + 2 * pf - kf) // stride_f + 1
    cols = np.zeros((C, kf, kt, Fo, T), np.float32)
    for a in range(kf):
        for b in range(kt):
            cols[:, a, b] = xp[:, a:a + stride_f * (Fo - 1) + 1:stride_f, b:b + T]
    y = w.reshape(O, -1) @ cols.reshape(C * kf * kt, Fo * T)
    return y.reshape(O, Fo, T).astype(np.float32)


def _relu(x):
    return np.maximum(x, 0.0).astype(np.float32)


def campplus(feats: np.ndarray, W: dict) -> np.ndarray:
    """feats [T][80] -> embedding [512] (wespeaker CAMPPlus forward, eval mode)."""
    x = feats.T[None].astype(np.float32)                                  # [1][80][T]
    out = _relu(_affine(_conv2d(x, W["head.conv1"]), W, "head.bn1"))
    for L in (1, 2):
        for b in range(2):
            p = "head.layer%d.%d" % (L, b)
            s = 2 if b == 0 else 1
            y = _relu(_affine(_conv2d(out, W[p + ".conv1"], s), W, p + ".bn1"))
            y = _affine(_conv2d(y, W[p + ".conv2"]), W, p + ".bn2")
            sc = _affine(_conv2d(out, W[p + ".shortcut"], 2), W, p + ".shortcut_bn") if b == 0 else out
            out = _relu(y + sc)
    out = _relu(_affine(_conv2d(out, W["head.conv2"], 2), W, "head.bn2"))   # [32][10][T]
    C, F, T = out.shape
    x = out.reshape(C * F, T)
    x = _relu(_affine(_conv1d(x, W["tdnn.linear"], None, stride=2, pad=2), W, "tdnn.bn"))
    for bi, (nl, k, dil) in enumerate(CAM_BLOCKS):
        for li in range(nl):
            p = "block%d.%d" % (bi + 1, li)
            h = _relu(_affine(x, W, p + ".bn1"))
            h = _conv1d(h, W[p + ".linear1"])
            h = _relu(_affine(h, W, p + ".bn2"))
            y = _conv1d(h, W[p + ".local"], None, pad=(k - 1) // 2 * dil, dil=dil)
            Tn = h.shape[1]
            ctx = h.mean(1, keepdims=True, dtype=np.float64).astype(np.float32)
            nseg = (Tn + 99) // 100
            seg = np.stack([h[:, s * 100:min(Tn, s * 100 + 100)].mean(1, dtype=np.float64) for s in range(nseg)], 1)
            seg = np.repeat(seg.astype(np.float32), 100, axis=1)[:, :Tn]
            c = ctx + seg
            c = _relu(_conv1d(c, W[p + ".cam1.weight"], W[p + ".cam1.bias"]))
            m = (1.0 / (1.0 + np.exp(-_conv1d(c, W[p + ".cam2.weight"], W[p + ".cam2.bias"])))).astype(np.float32)
            x = np.concatenate([x, (y * m).astype(np.float32)], 0)
        x = _relu(_affine(x, W, "transit%d.bn" % (bi + 1)))
        x = _conv1d(x, W["transit%d.linear" % (bi + 1)])
    x = _relu(_affine(x, W, "out.bn"))
    mean = x.mean(1, dtype=np.float64)
    std = x.std(1, ddof=1, dtype=np.float64) if x.shape[1] > 1 else np.full(x.shape[0], np.nan)
    st = np.concatenate([mean, std]).astype(np.float32)
    e = (W["dense.linear"].reshape(512, -1) @ st).astype(np.float32)
    return (e * W["dense.bn.scale"] + W["dense.bn.shift"]).astype(np.float32)


def compute_embedding(samples_i16: np.ndarray, W: dict | None = None):
    """EmbeddingExtractor::compute; None where the reference's ORT call errors (no frames)."""
    W = W if W is not None else cam_weights()
    f = compute_feats(samples_i16)
    if f.shape[0] == 0:
        return None
    return campplus(f, W)


# ------------------------------------------------------------------ a19 EmbeddingManager
class EmbeddingManager:
    """pyannote_rs::EmbeddingManager (speaker ids from 1; embeddings never updated).  Rust
    HashMap iteration order only matters on exact ties; ids are visited in ascending order."""

    def __init__(self, max_speakers: int):
        self.max_speakers = max_speakers
        self.speakers = {}
        self.next_id = 1

    @staticmethod
    def cosine(a, b):
        a = np.asarray(a, np.float32)
        b = np.asarray(b, np.float32)
        return np.float32(np.float32(a @ b) / (np.float32(np.sqrt(np.float32(a @ a))) * np.float32(np.sqrt(np.float32(b @ b)))))

    def search_speaker(self, emb, threshold: float):
        best, best_sim = None, np.float32(threshold)
        for sid in sorted(self.speakers):
            s = self.cosine(emb, self.speakers[sid])
            if s > best_sim:
                best, best_sim = sid, s
        if best is None and len(self.speakers) < self.max_speakers:
            sid = self.next_id
            self.speakers[sid] = np.asarray(emb, np.float32)
            self.next_id += 1
            return sid
        return best

    def get_best_speaker_match(self, emb):
        if not self.speakers:
            return None
        best, best_sim = 0, np.float32(-np.inf)
        for sid in sorted(self.speakers):
            s = self.cosine(emb, self.speakers[sid])
            if s > best_sim:
                best, best_sim = sid, s
        return best

    def assign(self, emb, threshold: float) -> str:
        """src/transcribe.rs:478-497."""
        if emb is None:
            return "?"
        if len(self.speakers) == self.max_speakers:
            r = self.get_best_speaker_match(emb)
        else:
            r = self.search_speaker(emb, threshold)
        return "?" if r is None else str(r)
