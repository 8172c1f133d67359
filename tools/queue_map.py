"""Which kernels share a hardware queue (rocprofv3 kernel trace, Queue_Id / Stream_Id columns).

HIP multiplexes a process's streams onto a few hardware queues per priority level; a queue runs
its packets in order, so a kernel on the step batcher's queue that belongs to another stream
delays every batched step queued behind it.  Per queue: dispatches, summed duration, streams,
and the kernel families on it; on the queues that carry decoder-rows kernels (the batcher's, the
DTW queue's) also per stream, and the summed time of the queue's idle gaps between consecutive
dispatches of the queue's main stream that another stream's kernel started in.
With a memory-copy trace beside it (rocprofv3 --memory-copy-trace): copies per direction.

Usage: python tools/queue_map.py run_kernel_trace.csv [label] [run_memory_copy_trace.csv]
"""
import collections
import csv
import re
import sys


def family(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"<.*", "", n)
    return n.replace("void ", "").replace("wdr::", "").strip()


def main():
    path = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else path
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r.get("Queue_Id", "?"), r.get("Stream_Id", "?"), family(r.get("Kernel_Name", "")),
                         int(r.get("Start_Timestamp", 0)), int(r.get("End_Timestamp", 0))))
    q = collections.defaultdict(lambda: dict(n=0, ns=0, streams=collections.Counter(), fam=collections.Counter(),
                                             fam_ns=collections.Counter(), per=collections.defaultdict(collections.Counter)))
    for qid, sid, nm, t0, t1 in rows:
        e = q[qid]
        e["n"] += 1
        e["ns"] += t1 - t0
        e["streams"][sid] += t1 - t0
        e["fam"][nm] += 1
        e["fam_ns"][nm] += t1 - t0
        e["per"][sid][nm] += 1
    print("== %s: %d queues" % (label, len(q)))
    for qid, e in sorted(q.items(), key=lambda kv: -kv[1]["ns"]):
        tag = "  <- decoder rows" if e["fam"].get("k_skinny", 0) else ""
        print("queue %s: %d dispatches, %.3f s, %d streams%s" % (qid, e["n"], e["ns"] * 1e-9, len(e["streams"]), tag))
        for nm, ns in e["fam_ns"].most_common(8):
            print("    %-28s %7d  %8.1f ms" % (nm[:28], e["fam"][nm], ns * 1e-6))
        if tag:
            main_sid = max(e["per"], key=lambda s: e["per"][s].get("k_skinny", 0))
            for sid, ns in e["streams"].most_common():
                c = e["per"][sid]
                print("    stream %-6s %8.1f ms  %6d dispatches  %s" % (
                    sid, ns * 1e-6, sum(c.values()), ", ".join("%s %d" % kv for kv in c.most_common(4))))
            # other streams' kernels that ran inside the main stream's gaps on this queue
            ev = sorted((t0, t1, sid) for qq, sid, nm, t0, t1 in rows if qq == qid)
            other = [(t0, t1) for t0, t1, sid in ev if sid != main_sid]
            print("    other streams' kernel time on this queue: %.1f ms in %d dispatches" % (
                sum(t1 - t0 for t0, t1 in other) * 1e-6, len(other)))
    if len(sys.argv) > 3:
        cp = collections.defaultdict(lambda: [0, 0, 0])
        with open(sys.argv[3]) as f:
            for r in csv.DictReader(f):
                k = r.get("Direction", r.get("Operation", "?"))
                cp[k][0] += 1
                cp[k][1] += int(r.get("End_Timestamp", 0)) - int(r.get("Start_Timestamp", 0))
                cp[k][2] += int(r.get("Bytes", r.get("Size", 0)) or 0)
        for k, (n, ns, b) in sorted(cp.items()):
            print("copies %-24s %6d  %8.1f ms  %10.1f MB" % (k, n, ns * 1e-6, b / 1e6))


if __name__ == "__main__":
    main()
