"""Summarise a tools/profile.sh run into profiles/ (tracked):
  profiles/<tag>_kernel_stats.csv   copy of rocprofv3 --stats kernel summary
  profiles/<tag>_pmc.json           per-launch FETCH_SIZE / WRITE_SIZE of the render kernel
  profiles/traffic_<tag>.json       HBM bytes per launch, read by bench.py (roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB,
collected in separate --pmc passes; on gfx950 FETCH_SIZE reports half the bytes
of wide coalesced reads, so reads are doubled (the guide calibrates that factor
for 16-B streaming loads only; our 4-B gathers are uncalibrated and the raw
value is kept beside it).
"""
import csv
import json
import os
import shutil
import statistics
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = sys.argv[2] if len(sys.argv) > 2 else f"gpurun_out/prof_{tag}"
cfg = sys.argv[3] if len(sys.argv) > 3 else "C3"
cam = sys.argv[4] if len(sys.argv) > 4 else "K1"
flags = int(sys.argv[5]) if len(sys.argv) > 5 else 48          # VX_FLAG_FULL_QUALITY
samples = int(sys.argv[6]) if len(sys.argv) > 6 else 1
# the bench's timed kernel: RGBA8, no stats, untiled; EXT instantiation unless v1
# EXT mode 0 v1 / 1 extensions / 2 soft shadows; either primary-index
# instantiation (the last template argument is left open)
KERNEL = f"k_render<1, false, false, {2 if samples > 1 else (1 if flags & 0x30 else 0)},"
os.makedirs("profiles", exist_ok=True)
shutil.copy(f"{src}/trace/run_kernel_stats.csv", f"profiles/{tag}_kernel_stats.csv")


def counter(path, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if KERNEL in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    return vals


fetch = counter(f"{src}/fetch/run_counter_collection.csv", "FETCH_SIZE")
write = counter(f"{src}/write/run_counter_collection.csv", "WRITE_SIZE")
avg_ns = None
with open(f"{src}/trace/run_kernel_stats.csv") as f:
    for row in csv.DictReader(f):
        if KERNEL in row["Name"]:
            avg_ns = float(row["AverageNs"])
fk, wk = statistics.median(fetch), statistics.median(write)
raw = (fk + wk) * 1024
corr = (2 * fk + wk) * 1024
pmc = {"kernel": KERNEL, "launches": [len(fetch), len(write)], "FETCH_SIZE_KiB_median": fk,
       "WRITE_SIZE_KiB_median": wk, "hbm_bytes_raw": raw, "hbm_bytes_read_x2": corr, "avg_duration_ns": avg_ns}
json.dump(pmc, open(f"profiles/{tag}_pmc.json", "w"), indent=1)
json.dump({"config": cfg, "camera": cam, "flags": flags, "samples": samples,
           "hbm_bytes_per_launch": int(corr), "hbm_bytes_raw": int(raw),
           "source": f"profiles/{tag}_pmc.json"}, open(f"profiles/traffic_{tag}.json", "w"), indent=1)
print(json.dumps(pmc, indent=1))
