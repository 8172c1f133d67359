#!/usr/bin/env python3
"""Batched-step timeline from a rocprofv3 kernel trace of bench.py (WDR_LAUNCH_LOCK=1): on the
step batcher's stream (the one with the most k_embed dispatches: every rows forward starts with
one), per step: span, sum of its kernel durations, and the gaps between its kernels -- for all
steps and split into decode-only steps and mixed ones (a prompt prefill / DTW re-forward rides
along: MFMA cross-attention tiles present); and what the rest of the GPU ran during those gaps
and during the step kernels (kernel classes by overlap time).
usage: step_gaps.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
cnt = collections.Counter(r["Stream_Id"] for r in rows if "k_embed" in r["Kernel_Name"])
bs = cnt.most_common(1)[0][0]
mine = sorted((r for r in rows if r["Stream_Id"] == bs), key=lambda r: r["s"])
others = sorted((r for r in rows if r["Stream_Id"] != bs), key=lambda r: r["s"])
steps, cur = [], None
for r in mine:
    if "k_embed" in r["Kernel_Name"]:
        cur = []
        steps.append(cur)
    if cur is not None:
        cur.append(r)
span = ksum = gap = 0.0
gaps = []
for st in steps:
    span += (st[-1]["e"] - st[0]["s"]) / 1e3
    ksum += sum(r["e"] - r["s"] for r in st) / 1e3
    for a, b in zip(st, st[1:]):
        if b["s"] > a["e"]:
            gaps.append((a["e"], b["s"], b["Kernel_Name"]))
gap = sum(b - a for a, b, _ in gaps) / 1e3
n = max(1, len(steps))
print("batcher stream %s: %d steps, span %.1f us/step, kernels %.1f us/step, gaps %.1f us/step, %.1f kernels/step"
      % (bs, len(steps), span / n, ksum / n, gap / n, sum(len(s) for s in steps) / n))
for name, sel in (("decode-only", [st for st in steps if not any("k_xattn_mma" in r["Kernel_Name"] for r in st)]),
                  ("mixed", [st for st in steps if any("k_xattn_mma" in r["Kernel_Name"] for r in st)])):
    if not sel:
        continue
    m = len(sel)
    sp = sum((st[-1]["e"] - st[0]["s"]) / 1e3 for st in sel) / m
    ks = sum(sum(r["e"] - r["s"] for r in st) / 1e3 for st in sel) / m
    print("  %-11s %5d steps: span %.1f us, kernels %.1f us, gaps %.1f us, %.1f kernels/step"
          % (name, m, sp, ks, sp - ks, sum(len(st) for st in sel) / m))


def cls(name):
    for k in ("k_gemm4", "k_gemm5", "k_gemm2", "k_gemm32", "k_gemm<", "k_flash", "k_skinny", "k_mgemv", "k_dgemv", "k_xattn",
              "k_dec_self", "layernorm", "k_ln_rows", "k_lstm", "k_fbank", "k_mel", "k_dtw", "k_aheads",
              "copyBuffer", "k_logits", "k_cam"):
        if k in name:
            return k
    return "other"


# overlap of other streams' kernels with the gaps (two-pointer sweep, both sorted by start)
ov = collections.Counter()
j0 = 0
for a, b, _ in gaps:
    while j0 < len(others) and others[j0]["e"] < a - 2_000_000:
        j0 += 1
    j = j0
    while j < len(others) and others[j]["s"] < b:
        o = others[j]
        x = min(b, o["e"]) - max(a, o["s"])
        if x > 0:
            ov[cls(o["Kernel_Name"])] += x / 1e3
        j += 1
# other streams' kernels overlapping the step kernels themselves
ovk = collections.Counter()
kints = sorted((r["s"], r["e"]) for st in steps for r in st)
j0 = 0
for a, b in kints:
    while j0 < len(others) and others[j0]["e"] < a - 2_000_000:
        j0 += 1
    j = j0
    while j < len(others) and others[j]["s"] < b:
        o = others[j]
        x = min(b, o["e"]) - max(a, o["s"])
        if x > 0:
            ovk[cls(o["Kernel_Name"])] += x / 1e3
        j += 1
print("step kernel time overlapped by other streams' kernels (us per step):")
for k, v in ovk.most_common(12):
    print("  %-12s %8.1f" % (k, v / n))
busy = collections.Counter()
for st in steps:
    for r in st:
        busy[cls(r["Kernel_Name"])] += (r["e"] - r["s"]) / 1e3
print("gap time overlapped by other streams' kernels (us per step):")
for k, v in ov.most_common(12):
    print("  %-12s %8.1f" % (k, v / n))
print("step kernel time by class (us per step):")
for k, v in busy.most_common(12):
    print("  %-12s %8.1f" % (k, v / n))
# gap length distribution by the kernel that followed
byk = collections.defaultdict(list)
for a, b, k in gaps:
    byk[cls(k)].append((b - a) / 1e3)
print("gap before kernel class: count, mean us, p90 us")
for k, v in sorted(byk.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print("  %-12s %6d %7.1f %7.1f" % (k, len(v), sum(v) / len(v), v[int(0.9 * (len(v) - 1))]))
