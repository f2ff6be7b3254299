"""Summarise rocprofv3 --pmc counter_collection CSVs: mean value per counter per kernel."""
import collections
import csv
import glob
import os
import sys

vals = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0][-60:]
            vals[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:60s} {c:28s} n={len(v):3d} mean={sum(v)/len(v):.6g}")
