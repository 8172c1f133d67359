#!/usr/bin/env python3
"""GPU busy fraction (union of kernel intervals) and per-group busy share over the timed region
of a rocprofv3 kernel trace: busy.py <kernel_trace.csv> [t_from_frac]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
frac0 = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
t0 = t0 + int((t1 - t0) * frac0)
iv = [x for x in iv if x[0] >= t0]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
print("span %.3f s, busy %.3f s (%.1f%%), kernels %d, sum of durations %.3f s (mean concurrency %.2f)"
      % (span / 1e9, busy / 1e9, 100 * busy / span, len(iv), sum(e - s for s, e, _ in iv) / 1e9,
         sum(e - s for s, e, _ in iv) / max(busy, 1)))
