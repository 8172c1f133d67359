#!/usr/bin/env python3
"""Summary of a WDR_BATCH_LOG file (StepBatcher launches: start s, rows, wall ms[, prefill rows,
DTW rows, GPU span ms, host enqueue ms]): rows histogram with the wall time spent at each row count, decode-only (graph
replay) vs mixed (eager: a prefill or DTW re-forward rides along) launches, the host gap
between one launch's end and the next one's start, and launches per tenth of the run.
usage: batch_log.py <log> [t0_gap_s]"""
import collections
import sys

L = []
for ln in open(sys.argv[1]):
    f = ln.split()
    if not f:
        continue
    t, r, w = float(f[0]), int(f[1]), float(f[2])
    pre = int(f[3]) if len(f) > 3 else 0
    dtw = int(f[4]) if len(f) > 4 else 0
    g = float(f[5]) if len(f) > 5 else 0.0
    q = float(f[6]) if len(f) > 6 else 0.0
    L.append((t, r, w, pre, dtw, g, q))
# the bench runs a warmup pass then the timed one: split at the largest gap between launches
gaps = [(L[i + 1][0] - L[i][0], i + 1) for i in range(len(L) - 1)]
cut = max(gaps)[1] if gaps and max(gaps)[0] > float(sys.argv[2] if len(sys.argv) > 2 else 0.5) else 0
L = L[cut:]
t0, t1 = L[0][0], L[-1][0] + L[-1][2] / 1e3
rows = sum(x[1] for x in L)
print("launches %d rows %d (%.2f per launch) span %.3f s, in steps %.3f s"
      % (len(L), rows, rows / len(L), t1 - t0, sum(x[2] for x in L) / 1e3))
host_gap = sum(max(0.0, L[i + 1][0] - (L[i][0] + L[i][2] / 1e3)) for i in range(len(L) - 1))
print("host gaps between launches %.3f s (%.1f us per launch)" % (host_gap, host_gap * 1e6 / max(1, len(L) - 1)))
for name, sel in (("decode-only (graph)", [x for x in L if x[3] == 0 and x[4] == 0]),
                  ("mixed (eager)", [x for x in L if x[3] or x[4]])):
    if sel:
        print("%-20s launches %5d  rows %7.2f  ms/launch %7.3f (GPU span %7.3f, host enqueue %7.3f)  wall %.3f s  prefill rows %d  DTW rows %d"
              % (name, len(sel), sum(x[1] for x in sel) / len(sel), sum(x[2] for x in sel) / len(sel),
                 sum(x[5] for x in sel) / len(sel), sum(x[6] for x in sel) / len(sel), sum(x[2] for x in sel) / 1e3, sum(x[3] for x in sel),
                 sum(x[4] for x in sel)))
h = collections.defaultdict(lambda: [0, 0.0])
for _, r, w, _, _, _, _ in L:
    h[(r + 7) // 8 * 8][0] += 1
    h[(r + 7) // 8 * 8][1] += w
print("rows<=  launches  wall_s  ms/launch")
for r in sorted(h):
    n, w = h[r]
    print("%5d %9d %7.3f %9.3f" % (r, n, w / 1e3, w / n))
print("by tenth of the span: launches, mean rows, mean ms")
for k in range(10):
    a, b = t0 + (t1 - t0) * k / 10, t0 + (t1 - t0) * (k + 1) / 10
    sel = [(x[1], x[2]) for x in L if a <= x[0] < b]
    if sel:
        print("  %d: %5d %6.2f %7.3f" % (k, len(sel), sum(r for r, _ in sel) / len(sel), sum(w for _, w in sel) / len(sel)))
