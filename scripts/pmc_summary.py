"""Summarise rocprofv3 --pmc CSV passes (scripts/pmc.sh output) per kernel,
per dispatch (sums divided by the number of dispatches)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sorted(glob.glob(d + "/p*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, c in agg.items():
    print(k)
    for name, v in sorted(c.items()):
        n = len(disp[(k, name)])
        print("  %-24s %16.4g   (per dispatch, %d dispatches)" % (name, v / n, n))
