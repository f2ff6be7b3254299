"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_<tag>.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (both reported in KiB); the factor 2 is
the gfx950 correction from MI355X_MICROARCH.md (FETCH_SIZE reports half of a wide coalesced
streaming read; WRITE_SIZE is exact for 16-B-per-lane stores).

usage: python scripts/pmc_traffic.py TAG KERNEL_SUBSTRING PMC_DIR [PMC_DIR ...]
"""
import collections
import csv
import glob
import json
import os
import sys

tag, needle, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
vals = collections.defaultdict(list)
kname = None
for d in dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if needle not in r["Kernel_Name"]:
                continue
            kname = r["Kernel_Name"]
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
    sys.exit(f"no FETCH_SIZE/WRITE_SIZE samples for kernels matching {needle!r}")
mean = {k: sum(v) / len(v) for k, v in vals.items()}
out = {
    "kernel": kname,
    "launches": {k: len(v) for k, v in vals.items()},
    "fetch_size_kib": mean["FETCH_SIZE"],
    "write_size_kib": mean["WRITE_SIZE"],
    "hbm_bytes_per_launch": (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024,
    "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace), "
              "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB per MI355X_MICROARCH.md gfx950 correction",
}
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(root, "profiles", f"pmc_{tag}.json")
os.makedirs(os.path.dirname(path), exist_ok=True)
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out))
