#!/usr/bin/env python3
"""Shrink a rocprofv3 output directory in place: keep only the rows of the
coding kernels (Kernel_Name containing 'ec_') in the kernel-trace and
counter-collection CSVs, so a profiling session's gpurun_out stays far below
the 64 MiB that gpurun copies back (bench.py's data generation launches
thousands of small torch kernels).  Usage: prof_filter.py DIR [PATTERN]"""
import csv
import os
import sys


def main():
    top = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "ec_"
    for root, _, files in os.walk(top):
        for f in files:
            p = os.path.join(root, f)
            if not f.endswith(".csv") or not ("kernel_trace" in f or "counter_collection" in f):
                continue
            with open(p, newline="") as fh:
                rows = list(csv.reader(fh))
            if not rows:
                continue
            hdr = rows[0]
            col = hdr.index("Kernel_Name") if "Kernel_Name" in hdr else None
            keep = [r for r in rows[1:] if col is None or pat in r[col]]
            with open(p, "w", newline="") as fh:
                w = csv.writer(fh)
                w.writerow(hdr)
                w.writerows(keep)


if __name__ == "__main__":
    main()
