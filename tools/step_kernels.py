#!/usr/bin/env python3
"""Per-kernel time per batched step by row count, from a rocprofv3 kernel trace of
tools/batch_probe.py (WDR_NO_GRAPH=1): usage step_kernels.py <run_kernel_trace.csv> [iters] [R,..]"""
import collections
import csv
import sys

path = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
show = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,4,8").split(",")]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
bs = rows[-1]["Stream_Id"]
steps, cur = [], None
for r in rows:
    if r["Stream_Id"] != bs:
        continue
    if "k_embed" in r["Kernel_Name"]:
        cur = []
        steps.append(cur)
    if cur is not None:
        cur.append(r)
per = iters + 1
for i in range(len(steps) // per):
    R = i + 1
    ss = steps[i * per + 1:(i + 1) * per]
    agg = collections.defaultdict(lambda: [0, 0.0])
    span = 0.0
    for st in ss:
        span += (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3
        for r in st:
            a = agg[r["Kernel_Name"].split("(")[0]]
            a[0] += 1
            a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(v[1] for v in agg.values()) / len(ss)
    print("R=%d  step span %.1f us, kernel sum %.1f us" % (R, span / len(ss), tot))
    if R in show:
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:10]:
            print("   %8.1f us/step  n=%3d avg %6.2f  %s" % (v[1] / len(ss), v[0] // len(ss), v[1] / v[0], k[:100]))
