#!/usr/bin/env python3
"""Summarise tools/kbench/xover_cells.sh logs: per cell the GPU-only, CPU-only
and auto rates, auto / max(GPU, CPU), and the median.  Usage: FILE..."""
import re
import statistics
import sys


def main():
    for path in sys.argv[1:]:
        cells = {}
        for line in open(path):
            m = re.match(r"(\w+)\s+(\S+)\s+(\w+)\s+(\w+)\s+(\d+) KiB x\s+(\d+) thr:\s+([\d.]+) GB/s"
                         r".*\[(.*)\]", line)
            if not m:
                continue
            mode, geo, op, _, kib, thr, gb, st = m.groups()
            cells.setdefault((geo, op, int(kib), int(thr)), {})[mode] = (float(gb), st)
        ratios = []
        print("==", path)
        for key, v in cells.items():
            if len(v) < 3:
                continue
            best = max(v["gpu"][0], v["cpu"][0])
            r = v["auto"][0] / best
            ratios.append(r)
            print("%-5s %-3s %6d x%-2d gpu %7.2f cpu %7.2f auto %7.2f  %.2f %s%s" % (
                key + (v["gpu"][0], v["cpu"][0], v["auto"][0], r, v["auto"][1].split(":", 1)[1],
                       "  <--" if r < 0.9 else "")))
        if ratios:
            print("median %.3f  below 0.9: %d of %d" % (statistics.median(ratios),
                                                       sum(r < 0.9 for r in ratios), len(ratios)))


if __name__ == "__main__":
    main()
