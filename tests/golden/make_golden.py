"""Generate the golden fixtures that pin the oracle (run once in the build container).

Source of truth for generic math: transformers 5.15.0 (installed here; the
reference's own whisper.cpp / ggml sources are not in the container, SURVEY.md
§8(c)).  Outputs (small .npz data files only — inputs and expected outputs):

  mel_filters.npz   transformers.audio_utils.mel_filter_bank slaney 80 / 128 bins
  power_spec.npz    transformers.audio_utils.spectrogram (periodic hann, 400/160, power 2)
  dtw_cases.npz     transformers ... generation_whisper._dynamic_time_warping,
                    incl. integer-valued matrices full of ties
  medfilt.npz       transformers ... generation_whisper._median_filter (width 7, reflect)
  kaldi_fbank.npz   transformers.audio_utils.spectrogram with Kaldi settings (povey, 0.97,
                    DC removal, 512-pt, kaldi mel 20..8000 Hz, log, FLT_EPSILON floor)
  pyannote_seg.npz  segmentation-3.0 structure in torch ops (nn.LSTM etc.), oracle weights
  campplus.npz      CAM++ structure in torch ops (conv2d strides, avg_pool1d ceil_mode), oracle weights
  whisper_tiny.npz  WhisperModel (eager attention, activation 'gelu_new') loaded with the
                    synthetic 'tiny-test' weights: encoder output rows and decoder logits

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))


def main():
    import torch
    from transformers.audio_utils import mel_filter_bank, spectrogram, window_function
    from transformers.models.whisper.generation_whisper import _dynamic_time_warping, _median_filter

    rng = np.random.default_rng(1234)

    # ---- mel filters
    fb = {}
    for n in (80, 128):
        f = mel_filter_bank(num_frequency_bins=201, num_mel_filters=n, min_frequency=0.0, max_frequency=8000.0,
                            sampling_rate=16000, norm="slaney", mel_scale="slaney")
        fb["f%d" % n] = f.T.astype(np.float32)            # [n_mels][201]
    np.savez_compressed(os.path.join(HERE, "mel_filters.npz"), **fb)

    # ---- power spectrum of a few frames
    x = (rng.standard_normal(400 + 160 * 7) * 0.1).astype(np.float32)
    win = window_function(400, "hann", periodic=True)
    spec = spectrogram(x.astype(np.float64), win, frame_length=400, hop_length=160, power=2.0, center=False)
    np.savez_compressed(os.path.join(HERE, "power_spec.npz"), x=x, power=spec.T.astype(np.float64))  # [frames][201]

    # ---- DTW
    cases = {}
    shapes = [(3, 5), (5, 5), (7, 40), (12, 120), (30, 300)]
    for k, (n, m) in enumerate(shapes):
        a = rng.standard_normal((n, m)).astype(np.float32)
        ti, tj = _dynamic_time_warping(a)
        cases["x%d" % k], cases["ti%d" % k], cases["tj%d" % k] = a, ti.astype(np.int32), tj.astype(np.int32)
    for k, (n, m) in enumerate([(4, 9), (9, 30), (16, 64)]):
        a = rng.integers(-2, 3, size=(n, m)).astype(np.float32)   # lots of exact ties
        ti, tj = _dynamic_time_warping(a)
        kk = 100 + k
        cases["x%d" % kk], cases["ti%d" % kk], cases["tj%d" % kk] = a, ti.astype(np.int32), tj.astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "dtw_cases.npz"), **cases)

    # ---- median filter
    w = rng.standard_normal((2, 3, 50)).astype(np.float32)
    med = _median_filter(torch.from_numpy(w), 7).numpy()
    np.savez_compressed(os.path.join(HERE, "medfilt.npz"), x=w, y=med)

    # ---- Whisper layer math (f32 graph), synthetic tiny-test weights
    from transformers import WhisperConfig, WhisperModel
    from oracle.weights import hparams_for, synth_weights
    hp = hparams_for("tiny-test")
    W = synth_weights(hp, std=0.02, emb_std=0.2)
    cfg = WhisperConfig(vocab_size=hp.n_vocab, num_mel_bins=hp.n_mels, encoder_layers=hp.n_audio_layer,
                        encoder_attention_heads=hp.n_audio_head, decoder_layers=hp.n_text_layer,
                        decoder_attention_heads=hp.n_text_head, d_model=hp.n_audio_state,
                        encoder_ffn_dim=4 * hp.n_audio_state, decoder_ffn_dim=4 * hp.n_text_state,
                        max_source_positions=hp.n_audio_ctx, max_target_positions=hp.n_text_ctx,
                        activation_function="gelu_new", dropout=0.0, attention_dropout=0.0,
                        activation_dropout=0.0, scale_embedding=False)
    cfg._attn_implementation = "eager"
    model = WhisperModel(cfg).eval()
    sd = {}
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    sd["encoder.conv1.weight"] = T(W["encoder.conv1.weight"])
    sd["encoder.conv1.bias"] = T(W["encoder.conv1.bias"])
    sd["encoder.conv2.weight"] = T(W["encoder.conv2.weight"])
    sd["encoder.conv2.bias"] = T(W["encoder.conv2.bias"])
    sd["encoder.embed_positions.weight"] = T(W["encoder.positional_embedding"])
    for i in range(hp.n_audio_layer):
        p, q = f"encoder.blocks.{i}.", f"encoder.layers.{i}."
        sd[q + "self_attn.q_proj.weight"] = T(W[p + "attn.query.weight"])
        sd[q + "self_attn.q_proj.bias"] = T(W[p + "attn.query.bias"])
        sd[q + "self_attn.k_proj.weight"] = T(W[p + "attn.key.weight"])
        sd[q + "self_attn.v_proj.weight"] = T(W[p + "attn.value.weight"])
        sd[q + "self_attn.v_proj.bias"] = T(W[p + "attn.value.bias"])
        sd[q + "self_attn.out_proj.weight"] = T(W[p + "attn.out.weight"])
        sd[q + "self_attn.out_proj.bias"] = T(W[p + "attn.out.bias"])
        sd[q + "self_attn_layer_norm.weight"] = T(W[p + "attn_ln.weight"])
        sd[q + "self_attn_layer_norm.bias"] = T(W[p + "attn_ln.bias"])
        sd[q + "fc1.weight"] = T(W[p + "mlp.0.weight"])
        sd[q + "fc1.bias"] = T(W[p + "mlp.0.bias"])
        sd[q + "fc2.weight"] = T(W[p + "mlp.2.weight"])
        sd[q + "fc2.bias"] = T(W[p + "mlp.2.bias"])
        sd[q + "final_layer_norm.weight"] = T(W[p + "mlp_ln.weight"])
        sd[q + "final_layer_norm.bias"] = T(W[p + "mlp_ln.bias"])
    sd["encoder.layer_norm.weight"] = T(W["encoder.ln_post.weight"])
    sd["encoder.layer_norm.bias"] = T(W["encoder.ln_post.bias"])
    sd["decoder.embed_tokens.weight"] = T(W["decoder.token_embedding.weight"])
    sd["decoder.embed_positions.weight"] = T(W["decoder.positional_embedding"])
    for i in range(hp.n_text_layer):
        p, q = f"decoder.blocks.{i}.", f"decoder.layers.{i}."
        for a, b in (("attn", "self_attn"), ("cross_attn", "encoder_attn")):
            sd[q + b + ".q_proj.weight"] = T(W[p + a + ".query.weight"])
            sd[q + b + ".q_proj.bias"] = T(W[p + a + ".query.bias"])
            sd[q + b + ".k_proj.weight"] = T(W[p + a + ".key.weight"])
            sd[q + b + ".v_proj.weight"] = T(W[p + a + ".value.weight"])
            sd[q + b + ".v_proj.bias"] = T(W[p + a + ".value.bias"])
            sd[q + b + ".out_proj.weight"] = T(W[p + a + ".out.weight"])
            sd[q + b + ".out_proj.bias"] = T(W[p + a + ".out.bias"])
            sd[q + b + "_layer_norm.weight"] = T(W[p + a + "_ln.weight"])
            sd[q + b + "_layer_norm.bias"] = T(W[p + a + "_ln.bias"])
        sd[q + "fc1.weight"] = T(W[p + "mlp.0.weight"])
        sd[q + "fc1.bias"] = T(W[p + "mlp.0.bias"])
        sd[q + "fc2.weight"] = T(W[p + "mlp.2.weight"])
        sd[q + "fc2.bias"] = T(W[p + "mlp.2.bias"])
        sd[q + "final_layer_norm.weight"] = T(W[p + "mlp_ln.weight"])
        sd[q + "final_layer_norm.bias"] = T(W[p + "mlp_ln.bias"])
    sd["decoder.layer_norm.weight"] = T(W["decoder.ln.weight"])
    sd["decoder.layer_norm.bias"] = T(W["decoder.ln.bias"])
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("k_proj.bias" in m for m in missing), missing
    for name, prm in model.named_parameters():
        if name.endswith("k_proj.bias"):
            prm.data.zero_()
    mel = (rng.standard_normal((1, hp.n_mels, 3000)) * 0.5).astype(np.float32)
    toks = np.array([[50257, 50363, 100, 2000, 30000]], np.int64)
    with torch.no_grad():
        out = model(input_features=torch.from_numpy(mel), decoder_input_ids=torch.from_numpy(toks),
                    output_attentions=True)
        enc = out.encoder_last_hidden_state[0].numpy()
        dec = out.last_hidden_state[0]
        logits = (dec @ model.decoder.embed_tokens.weight.T).numpy()
        cross = np.stack([a[0].numpy() for a in out.cross_attentions])   # [L][H][tok][1500]
    np.savez_compressed(os.path.join(HERE, "whisper_tiny.npz"), mel=mel[0], tokens=toks[0],
                        enc_rows=enc[::25], enc_sum=np.float64(enc.astype(np.float64).sum()),
                        logits_last=logits[-1].astype(np.float32), logits_top=np.argsort(-logits, axis=1)[:, :20],
                        cross_last=cross[-1].astype(np.float32))
    diarize_golden(np.random.default_rng(77))
    print("golden fixtures written to", HERE)


def diarize_golden(rng):
    """kaldi_fbank.npz / pyannote_seg.npz / campplus.npz: the diarization rows' generic math
    computed with transformers' Kaldi-compatible spectrogram and torch modules assembled with
    the oracle's synthetic weights (torch op semantics: InstanceNorm1d, MaxPool1d, the
    bidirectional nn.LSTM stack, Conv2d strides, avg_pool1d(ceil_mode) segment pooling,
    unbiased std) -- pins oracle/diarize.py against independent implementations."""
    import torch
    import torch.nn.functional as F
    from transformers.audio_utils import mel_filter_bank, spectrogram, window_function
    from oracle import diarize as D

    # ---- Kaldi fbank (SeamlessM4T / kaldi-compatible settings of transformers.audio_utils)
    x = (rng.standard_normal(16000 + 337) * 0.1).astype(np.float32)
    x += 0.3 * np.sin(2 * np.pi * 440 * np.arange(x.size) / 16000).astype(np.float32)
    mel = mel_filter_bank(num_frequency_bins=257, num_mel_filters=80, min_frequency=20, max_frequency=8000,
                          sampling_rate=16000, norm=None, mel_scale="kaldi", triangularize_in_mel_space=True)
    fb = spectrogram(x, window_function(400, "povey", periodic=False), frame_length=400, hop_length=160,
                     fft_length=512, power=2.0, center=False, preemphasis=0.97, mel_filters=mel, log_mel="log",
                     mel_floor=1.192092955078125e-07, remove_dc_offset=True).T
    np.savez_compressed(os.path.join(HERE, "kaldi_fbank.npz"), x=x, fbank=fb.astype(np.float32))

    torch.set_grad_enabled(False)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    # ---- segmentation-3.0 with torch modules
    W = D.seg_weights()
    win = np.zeros(160000, np.float32)
    pcm = (rng.standard_normal(120000) * 3000).astype(np.int16).astype(np.float32)
    win[:120000] = pcm
    def inorm(x, g, b):
        m = torch.nn.InstanceNorm1d(x.shape[1], affine=True)
        m.weight.copy_(T(g)); m.bias.copy_(T(b))
        return m(x)
    h = inorm(T(win)[None, None], W["wav_norm.weight"], W["wav_norm.bias"])
    h = torch.abs(F.conv1d(h, T(W["sinc.weight"]), stride=10))
    h = F.leaky_relu(inorm(F.max_pool1d(h, 3, 3), W["norm0.weight"], W["norm0.bias"]))
    h = F.conv1d(h, T(W["conv1.weight"]), T(W["conv1.bias"]))
    h = F.leaky_relu(inorm(F.max_pool1d(h, 3, 3), W["norm1.weight"], W["norm1.bias"]))
    h = F.conv1d(h, T(W["conv2.weight"]), T(W["conv2.bias"]))
    h = F.leaky_relu(inorm(F.max_pool1d(h, 3, 3), W["norm2.weight"], W["norm2.bias"]))
    lstm = torch.nn.LSTM(60, 128, num_layers=4, bidirectional=True, batch_first=True)
    for k, v in lstm.named_parameters():
        v.copy_(T(W["lstm." + k]))
    h, _ = lstm(h.transpose(1, 2))
    h = F.leaky_relu(F.linear(h, T(W["linear0.weight"]), T(W["linear0.bias"])))
    h = F.leaky_relu(F.linear(h, T(W["linear1.weight"]), T(W["linear1.bias"])))
    lp = torch.log_softmax(F.linear(h, T(W["classifier.weight"]), T(W["classifier.bias"])), -1)[0]
    np.savez_compressed(os.path.join(HERE, "pyannote_seg.npz"), win=win.astype(np.int16), logprobs=lp.numpy())

    # ---- CAM++ (wespeaker CAMPPlus structure) with torch ops
    CW = D.cam_weights()
    feats = (rng.standard_normal((237, 80)) * 2.0).astype(np.float32)
    bn = lambda x, n, dim=1: x * T(CW[n + ".scale"]).view(*([1] * dim), -1, *([1] * (x.dim() - dim - 1))) + \
        T(CW[n + ".shift"]).view(*([1] * dim), -1, *([1] * (x.dim() - dim - 1)))
    x = T(feats).T[None, None]                                     # [1][1][80][T]
    out = F.relu(bn(F.conv2d(x, T(CW["head.conv1"]), padding=1), "head.bn1"))
    for L in (1, 2):
        for b in range(2):
            p = "head.layer%d.%d" % (L, b)
            st = 2 if b == 0 else 1
            y = F.relu(bn(F.conv2d(out, T(CW[p + ".conv1"]), stride=(st, 1), padding=1), p + ".bn1"))
            y = bn(F.conv2d(y, T(CW[p + ".conv2"]), padding=1), p + ".bn2")
            sc = bn(F.conv2d(out, T(CW[p + ".shortcut"]), stride=(2, 1)), p + ".shortcut_bn") if b == 0 else out
            out = F.relu(y + sc)
    out = F.relu(bn(F.conv2d(out, T(CW["head.conv2"]), stride=(2, 1), padding=1), "head.bn2"))
    x = out.reshape(1, -1, out.shape[-1])
    x = F.relu(bn(F.conv1d(x, T(CW["tdnn.linear"]), stride=2, padding=2), "tdnn.bn"))
    for bi, (nl, k, dil) in enumerate(D.CAM_BLOCKS):
        for li in range(nl):
            p = "block%d.%d" % (bi + 1, li)
            hh = F.relu(bn(F.conv1d(F.relu(bn(x, p + ".bn1")), T(CW[p + ".linear1"])), p + ".bn2"))
            y = F.conv1d(hh, T(CW[p + ".local"]), padding=(k - 1) // 2 * dil, dilation=dil)
            seg = F.avg_pool1d(hh, kernel_size=100, stride=100, ceil_mode=True)
            seg = seg.unsqueeze(-1).expand(*seg.shape, 100).reshape(*seg.shape[:-1], -1)[..., :hh.shape[-1]]
            c = hh.mean(-1, keepdim=True) + seg
            c = F.relu(F.conv1d(c, T(CW[p + ".cam1.weight"]), T(CW[p + ".cam1.bias"])))
            m = torch.sigmoid(F.conv1d(c, T(CW[p + ".cam2.weight"]), T(CW[p + ".cam2.bias"])))
            x = torch.cat([x, y * m], 1)
        x = F.conv1d(F.relu(bn(x, "transit%d.bn" % (bi + 1))), T(CW["transit%d.linear" % (bi + 1)]))
    x = F.relu(bn(x, "out.bn"))
    stats = torch.cat([x.mean(-1), x.std(-1, unbiased=True)], -1)
    emb = F.conv1d(stats.unsqueeze(-1), T(CW["dense.linear"])).squeeze(-1)
    emb = emb * T(CW["dense.bn.scale"]) + T(CW["dense.bn.shift"])
    np.savez_compressed(os.path.join(HERE, "campplus.npz"), feats=feats, emb=emb[0].numpy())


if __name__ == "__main__":
    main()
