"""Development probe: average counters per kernel from tools/pmc_probe.sh."""
import collections
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "probe"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmc_%s_*/run_counter_collection.csv" % tag)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "ecdev" not in k:
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k[k.find("<"):k.find("(")])
    print("   " + "  ".join("%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(d.items())))
