#!/usr/bin/env python3
"""Per (kernel, grid size) averages of rocprofv3 --pmc counter_collection.csv files.

usage: pmc_kernels.py PMC_DIR [PMC_DIR ...] [--match SUBSTR]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                n = r.get("Kernel_Name", "")
                if a.match not in n:
                    continue
                key = (n.replace("void wdr::", "")[:40], r.get("Grid_Size", r.get("Grid_Size_X", "")))
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key in sorted(acc):
        c = acc[key]
        vals = "  ".join("%s=%.4g" % (k, sum(v) / len(v)) for k, v in sorted(c.items()))
        print("%-40s grid=%-8s %s" % (key[0], key[1], vals))
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = sum(c["TCC_HIT_sum"]), sum(c["TCC_MISS_sum"])
            print("%50s L2 hit rate %.3f" % ("", h / max(1.0, h + m)))


if __name__ == "__main__":
    main()
