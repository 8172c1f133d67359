#!/usr/bin/env python3
"""Summarise a rocprofv3 `--kernel-trace --stats --output-format csv` run directory.

Writes a per-kernel table (calls, total ms, avg us, share) and, per kernel class of bench.py's
live roofline (gemv / gemm / flash / xattn), the launch-weighted average duration so the two
can be compared.  Optionally folds in `--pmc FETCH_SIZE` / `WRITE_SIZE` counter_collection.csv
files (gfx950: FETCH_SIZE reports half the bytes of wide streaming reads -> doubled here,
MI355X_MICROARCH.md 'HBM').

usage: prof_summary.py TRACE_DIR [--fetch PMC_DIR] [--write PMC_DIR] [--top N] [--drop-trace]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

import re

# kernel classes (bench.py's live roofline classes plus the diarization stack): the encoder
# GEMMs are k_gemm / k_gemm2..5 / k_gemm8 / k_gemm8n -- NOT the f32 VALU k_gemm32 of CAM++ / segmentation
CLASSES = {
    "gemm": re.compile(r"\bk_gemm\d?n?[<(]"),
    "rows": re.compile(r"\bk_skinny<"),                       # decoder row projections (rows.h)
    "flash": re.compile(r"\bk_flash_attn(<\d+>)?\("),         # encoder self-attention
    "xattn": re.compile(r"\bk_xattn_(partial2?|mma)\b"),    # decoder cross-attention partials
    "diar": re.compile(r"\bk_(gemm32|lstm_scan|im2col_2d_b|im2col_1d_b|fbank|colstats_b|cam_|inorm|maxpool3|logsoftmax7)"),
}


def find(d, pat):
    got = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
    return got


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def classify(name):
    for c, rx in CLASSES.items():
        if rx.search(name):
            return c
    return None


def short(name, w=70):
    name = name.replace("void wdr::", "").replace("wdr::", "")
    return name if len(name) <= w else name[: w - 3] + "..."


def trace_table(d):
    per = defaultdict(lambda: [0, 0.0])
    for f in find(d, "*kernel_trace.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                n = col(r, "Kernel_Name", "Name")
                dt = int(col(r, "End_Timestamp")) - int(col(r, "Start_Timestamp"))
                per[n][0] += 1
                per[n][1] += dt
    return per


def pmc_table(d, counter):
    per = defaultdict(lambda: [0, 0.0])
    for f in find(d, "*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if col(r, "Counter_Name") != counter:
                    continue
                n = col(r, "Kernel_Name")
                per[n][0] += 1
                per[n][1] += float(col(r, "Counter_Value"))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--json", help="write per-class avg duration and PMC bytes/dispatch here (read by bench.py)")
    ap.add_argument("--drop-trace", action="store_true", help="delete the (large) per-dispatch trace csv afterwards")
    a = ap.parse_args()
    per = trace_table(a.trace_dir)
    tot = sum(v[1] for v in per.values()) or 1.0
    print("# per-kernel (rocprofv3 --kernel-trace), durations from the dispatch timestamps")
    print("%-70s %9s %11s %10s %6s" % ("kernel", "calls", "total_ms", "avg_us", "share"))
    for n, (c, ns) in sorted(per.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print("%-70s %9d %11.2f %10.3f %5.1f%%" % (short(n), c, ns / 1e6, ns / c / 1e3, 100 * ns / tot))
    print("total kernel time %.1f ms over %d dispatches" % (tot / 1e6, sum(v[0] for v in per.values())))
    print()
    print("# kernel classes of bench.py's live roofline")
    cls = defaultdict(lambda: [0, 0.0])
    for n, (c, ns) in per.items():
        k = classify(n)
        if k:
            cls[k][0] += c
            cls[k][1] += ns
    for k, (c, ns) in sorted(cls.items()):
        print("%-8s launches %8d  total %10.2f ms  avg %8.3f us  share %5.1f%%" % (k, c, ns / 1e6, ns / c / 1e3,
                                                                                  100 * ns / tot))
    out = {"total_kernel_ms": tot / 1e6,
           "classes": {k: {"launches": c, "avg_us": ns / c / 1e3, "total_ms": ns / 1e6, "share": ns / tot}
                       for k, (c, ns) in cls.items()}}
    for label, dd, counter, scale in (("FETCH_SIZE x2 (gfx950 correction)", a.fetch, "FETCH_SIZE", 2.0),
                                      ("WRITE_SIZE", a.write, "WRITE_SIZE", 1.0)):
        if not dd:
            continue
        pm = pmc_table(dd, counter)
        print()
        print("# %s, KB per dispatch" % label)
        pc = defaultdict(lambda: [0, 0.0])
        for n, (c, v) in sorted(pm.items(), key=lambda kv: -kv[1][1])[: a.top]:
            print("%-70s %9d %12.1f" % (short(n), c, scale * v / c))
        for n, (c, v) in pm.items():
            k = classify(n)
            if k:
                pc[k][0] += c
                pc[k][1] += scale * v
        for k, (c, v) in sorted(pc.items()):
            print("class %-8s %8d dispatches  %.1f KB/dispatch (x1024 B)" % (k, c, v / c))
            out["classes"].setdefault(k, {})[counter.lower() + "_bytes_per_dispatch"] = v / c * 1024.0
    if a.json:
        import json
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)
    if a.drop_trace:
        for f in find(a.trace_dir, "*kernel_trace.csv"):
            os.remove(f)


if __name__ == "__main__":
    main()
