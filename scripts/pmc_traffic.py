"""Turn rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE, and when present
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE) into profiles/pmc_<tag>.json.

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
# kernel durations from the passes' kernel traces (same kernels), for the effective clock
durs = []
for d in dirs:
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if needle in r.get("Kernel_Name", ""):
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
durs.sort()
out = {
    "kernel": kname,
    "launches": {k: len(v) for k, v in vals.items()},
    "fetch_size_kib": mean["FETCH_SIZE"],
    "write_size_kib": mean["WRITE_SIZE"],
    "hbm_bytes_per_launch": (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024,
    "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace), "
              "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB per MI355X_MICROARCH.md gfx950 correction",
}
if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
    gui = mean["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
    out["mfma_busy_frac"] = round(mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4 * gui), 4)
    if durs:
        out["effective_clock_ghz"] = round(gui / durs[len(durs) // 2], 3)
    out["method"] += ("; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (256 CU x 4 SIMD x GRBM_GUI_ACTIVE/8);"
                      " clock = GRBM_GUI_ACTIVE/8 / median profiled kernel duration")
if "SQ_INSTS_VALU" in mean and "SQ_INSTS_MFMA" in mean and mean["SQ_INSTS_MFMA"]:
    out["valu_insts_per_mfma"] = round(mean["SQ_INSTS_VALU"] / mean["SQ_INSTS_MFMA"], 2)
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(root, "profiles", f"pmc_{tag}.json")
os.makedirs(os.path.dirname(path), exist_ok=True)
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out))
