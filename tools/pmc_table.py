#!/usr/bin/env python3
"""Per-launch PMC averages from rocprofv3 --pmc runs (development tool).

Sums every counter over the rows of one dispatch (rocprofv3 may report a
counter per XCD / shader engine), then averages over the dispatches of each
kernel, skipping the first SKIP (default 5: the warm-up launches).

Usage: python tools/pmc_table.py DIR [DIR ...]   (each DIR holds
run_counter_collection.csv somewhere below it)"""
import collections
import csv
import glob
import os
import sys

SKIP = int(os.environ.get("SKIP", "5"))


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    kname = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
            kname[did] = r["Kernel_Name"]
    by_kernel = collections.defaultdict(list)
    for did in sorted(per):
        by_kernel[kname[did]].append(per[did])
    return by_kernel


def short(k):
    return k[k.find("ec_"):k.find("(")] if "ec_" in k else k[:80]


def main():
    for d in sys.argv[1:]:
        for k, rows in load(d).items():
            rows = rows[SKIP:] or rows
            names = sorted({c for r in rows for c in r})
            avg = {c: sum(r.get(c, 0.0) for r in rows) / len(rows) for c in names}
            print("%s  %s  (%d launches)" % (os.path.basename(d.rstrip("/")), short(k), len(rows)))
            print("    " + "  ".join("%s=%.4g" % (c, avg[c]) for c in names))


if __name__ == "__main__":
    main()
