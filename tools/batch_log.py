#!/usr/bin/env python3
"""Summary of a WDR_BATCH_LOG file (StepBatcher launches: start s, rows, wall ms): rows
histogram with the wall time spent at each row count, and launches per tenth of the run
(how the row count decays toward the tail).  usage: batch_log.py <log> [t0_gap_s]"""
import collections
import sys

L = [tuple(float(x) for x in ln.split()) for ln in open(sys.argv[1]) if ln.strip()]
# the bench runs a warmup pass then the timed one: split at the largest gap between launches
gaps = [(L[i + 1][0] - L[i][0], i + 1) for i in range(len(L) - 1)]
cut = max(gaps)[1] if gaps and max(gaps)[0] > float(sys.argv[2] if len(sys.argv) > 2 else 0.5) else 0
L = L[cut:]
t0, t1 = L[0][0], L[-1][0] + L[-1][2] / 1e3
print("launches %d rows %d (%.2f per launch) span %.3f s, in steps %.3f s"
      % (len(L), sum(r for _, r, _ in L), sum(r for _, r, _ in L) / len(L), t1 - t0, sum(w for *_, w in L) / 1e3))
h = collections.defaultdict(lambda: [0, 0.0])
for _, r, w in L:
    h[int(r)][0] += 1
    h[int(r)][1] += w
print("rows  launches  wall_s  ms/launch")
for r in sorted(h):
    n, w = h[r]
    print("%4d %9d %7.3f %9.3f" % (r, n, w / 1e3, w / n))
print("by tenth of the span: launches, mean rows, mean ms")
for k in range(10):
    a, b = t0 + (t1 - t0) * k / 10, t0 + (t1 - t0) * (k + 1) / 10
    sel = [(r, w) for t, r, w in L if a <= t < b]
    if sel:
        print("  %d: %5d %6.2f %7.3f" % (k, len(sel), sum(r for r, _ in sel) / len(sel), sum(w for _, w in sel) / len(sel)))
