#!/usr/bin/env python3
"""Summary of a WDR_CHAIN_LOG file (one line per State::full call of a multi-chain run: chain,
job, entry s, exit s, top_up ms, ready-wait ms, energy ms, decode ms, post ms): per chain and in
total, where a chain's wall goes -- inside its windows' decode loops (batched steps), in the
encode-ahead top_up (host launches), waiting for its encodes, the energy copy, the post-decode
host work, the rest of full() and the time between full() calls.  The last run of the file only
(from the last first call (job 0) of the chains on).  usage: chain_log.py <log>"""
import collections
import sys

L = []
for ln in open(sys.argv[1]):
    f = ln.split()
    if len(f) >= 9:
        L.append((int(f[0]), int(f[1]), float(f[2]), float(f[3])) + tuple(float(x) for x in f[4:9]) +
                 tuple(float(x) for x in f[9:11]))
L.sort(key=lambda x: x[2])
# the last run: from the latest first call (job 0) of every chain's last block on
last0 = {}
for x in L:
    if x[1] == 0:
        last0[x[0]] = x[2]
if last0:
    t_run = min(last0.values()) - 1e-6
    L = [x for x in L if x[2] >= t_run]
by = collections.defaultdict(list)
for x in L:
    by[x[0]].append(x)
tot = collections.Counter()
n_calls = 0
for c, xs in by.items():
    xs.sort(key=lambda x: x[2])
    wall = xs[-1][3] - xs[0][2]
    inside = sum(x[3] - x[2] for x in xs)
    tot["wall"] += wall
    tot["between calls"] += wall - inside
    for k, i in (("top_up", 4), ("ready wait", 5), ("energy", 6), ("decode loops", 7), ("post", 8),
                 ("  DTW-queue wait", 9), ("  encoder launch", 10)):
        tot[k] += sum(x[i] for x in xs if len(x) > i) / 1e3
    tot["rest of full"] += inside - sum(sum(x[4:9]) for x in xs) / 1e3
    n_calls += len(xs)
nc = max(1, len(by))
print("chains %d, calls %d; per chain (s) and per call (ms):" % (len(by), n_calls))
for k in ("wall", "decode loops", "top_up", "  DTW-queue wait", "  encoder launch", "ready wait", "energy", "post",
          "rest of full", "between calls"):
    print("  %-14s %7.3f s  %8.3f ms/call" % (k, tot[k] / nc, tot[k] * 1e3 / max(1, n_calls)))
# the tail: when each chain's last call ends, relative to the run's first call
t0 = min(xs[0][2] for xs in by.values())
ends = sorted(xs[-1][3] - t0 for xs in by.values())
if ends:
    print("chain ends (s after the run's first call): first %.3f, median %.3f, last %.3f; last - median %.3f s"
          % (ends[0], ends[len(ends) // 2], ends[-1], ends[-1] - ends[len(ends) // 2]))
    print("  " + " ".join("%.2f" % e for e in ends))
# the start: each chain's first call -- its ready wait is the wait for its first encode batch
firsts = sorted((xs[0][2] - t0 + xs[0][5] / 1e3, c) for c, xs in by.items())
if firsts:
    print("first decode (s after the run's first call, entry + ready wait of the chain's first call): "
          "first %.3f, median %.3f, last %.3f" % (firsts[0][0], firsts[len(firsts) // 2][0], firsts[-1][0]))
    print("  " + " ".join("%d:%.2f" % (c, t) for t, c in firsts))
    endc = {c: xs[-1][3] - t0 for c, xs in by.items()}
    print("ends by chain: " + " ".join("%d:%.2f" % (c, endc[c]) for c in sorted(endc)))
