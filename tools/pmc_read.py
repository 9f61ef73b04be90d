"""Average per-dispatch PMC counters of kernels matching a substring (rocprofv3 csv)."""
import csv
import glob
import sys
from collections import defaultdict

pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg, n = defaultdict(float), defaultdict(int)
for p in sorted(glob.glob(sys.argv[1] + "/*/run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / n[k]:16.1f}  (n={n[k]})")
