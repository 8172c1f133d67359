#!/usr/bin/env python3
"""Group a rocprofv3 kernel_stats.csv into pipeline stages (GPU time per stage)."""
import collections
import csv
import sys

GROUPS = [
    ("step-attn", ("k_dec_self_attn", "k_xattn_partial", "k_xattn_combine", "k_embed")),
    ("logits", ("k_logits",)),
    ("enc-gemm", ("k_gemm<", "k_gemm2<", "k_gemm3<", "k_gemm4<", "k_gemm5<", "k_gemm8<", "k_gemm8n<")),
    ("flash", ("k_flash",)),
    ("rows", ("k_skinny",)),
    ("layernorm", ("k_layernorm",)),
    ("dtw", ("k_dtw", "k_aheads")),
    ("mel", ("k_mel", "k_im2col", "k_energy", "k_i16")),
    ("diarize", ("k_fbank", "k_colstats", "k_lstm", "k_gemm32", "k_sinc", "k_seg", "k_cam", "k_tdnn", "k_bn",
                 "k_pool", "k_stats", "k_maxpool", "k_inorm", "k_lrelu", "k_head", "k_im2col2d")),
    ("vad", ("k_vad",)),
    ("copy", ("copyBuffer", "fillBuffer")),
]
rows = list(csv.DictReader(open(sys.argv[1])))
tot = collections.defaultdict(lambda: [0.0, 0])
for r in rows:
    name = r["Name"]
    g = next((g for g, keys in GROUPS if any(k in name for k in keys)), "other:" + name.split("(")[0][:40])
    tot[g][0] += float(r["TotalDurationNs"]) / 1e6
    tot[g][1] += int(r["Calls"])
all_ms = sum(v[0] for v in tot.values())
print("total kernel time %.1f ms" % all_ms)
for g, (ms, n) in sorted(tot.items(), key=lambda kv: -kv[1][0]):
    print("%-48s %9.1f ms %5.1f%%  %7d calls" % (g, ms, 100 * ms / all_ms, n))
