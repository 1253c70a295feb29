#!/usr/bin/env python3
"""Per-launch durations, in launch order, of the coding kernels in a
rocprofv3 --kernel-trace output directory (after prof_filter.py):
count, min / median / mean / max, and the sequence in groups of 10, so a
slow start, a drift under sustained load or outliers show.
Usage: [LAST=N] trace_seq.py DIR [PATTERN]"""
import csv
import os
import statistics
import sys


def main():
    top = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "ec_"
    rows = []
    for root, _, files in os.walk(top):
        for f in files:
            if f.endswith("kernel_trace.csv"):
                with open(os.path.join(root, f), newline="") as fh:
                    for r in csv.DictReader(fh):
                        if pat in r["Kernel_Name"]:
                            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                         r["Kernel_Name"]))
    rows.sort()
    by = {}
    for s, e, n in rows:
        by.setdefault(n, []).append((s, e))
    last = int(os.environ.get("LAST", "0"))        # only the last N launches of each kernel
    for n, v in by.items():
        if last:
            v = v[-last:]
        d = [(e - s) / 1e3 for s, e in v]
        gaps = [(v[i + 1][0] - v[i][1]) / 1e3 for i in range(len(v) - 1)]
        print("%s\n  launches %d  min %.1f  med %.1f  mean %.1f  max %.1f us; gap med %.1f us"
              % (n[:110], len(d), min(d), statistics.median(d), statistics.mean(d), max(d),
                 statistics.median(gaps) if gaps else 0.0))
        for i in range(0, len(d), 10):
            print("   " + " ".join("%6.1f" % x for x in d[i:i + 10]))


if __name__ == "__main__":
    main()
