"""Median per-dispatch counter values of the step kernel from tools/pmc.sh output."""
import collections
import csv
import glob
import statistics
import sys

out = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "core_"
agg = collections.defaultdict(list)
for f in glob.glob(f"{out}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"] and "reset" not in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    print(f"{k:32s} {statistics.median(agg[k]):16.1f}  (n={len(agg[k])})")
