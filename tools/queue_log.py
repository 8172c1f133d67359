"""Pair libwdr's stream creations (WDR_STREAM_LOG=1) with the HIP runtime's hardware-queue
choice printed just before each (AMD_LOG_LEVEL=3: 'acquireQueue refCount: Q (n)' for a new
queue, 'Selected queue refCount: Q (n)' for a shared one): which streams share which hardware
queue.  Usage: python tools/queue_log.py run.stderr"""
import collections
import re
import sys


def main():
    last_q = None
    q_of = []
    for line in open(sys.argv[1], errors="replace"):
        m = re.search(r"(acquireQueue|Selected queue) refCount: (0x[0-9a-f]+|\(nil\)|[0-9a-fx]+) \((\d+)\)", line)
        if m:
            last_q = m.group(2)
            continue
        if "Setting CU mask" in line:
            m2 = re.search(r"hardware queue (0x[0-9a-f]+)", line)
            last_q = (m2.group(1) if m2 else "?") + "(masked)"
            continue
        m = re.search(r"\[wdr-stream\] (\S+) (\S+)", line)
        if m:
            q_of.append((m.group(1), m.group(2), last_q))
            last_q = None
    by_q = collections.defaultdict(list)
    for what, s, q in q_of:
        by_q[q].append(what)
    for q, ws in by_q.items():
        c = collections.Counter(ws)
        print("%-28s %3d streams: %s" % (q, len(ws), ", ".join("%s x%d" % kv for kv in c.items())))
    print("creation order:", " ".join("%s@%s" % (w, (q or "?")[-6:]) for w, _, q in q_of[:60]))


if __name__ == "__main__":
    main()
