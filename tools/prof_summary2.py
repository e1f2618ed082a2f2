"""Summarise a tools/profile2.sh run into profiles/ (tracked; bench.py reads them):
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats kernel summary (the timed run)
  profiles/<tag>_pmc.json           per-launch medians of every counter of the render kernel
  profiles/traffic_<tag>.json       fabric bytes per launch (roofline.traffic)
  profiles/valu_<tag>.json          VALU issue utilisation etc. (roofline.valu)

Fabric bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB
from separate passes; gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so reads are doubled (the guide calibrates that for 16-B
loads; the raw sum is kept beside it).  VALU issue: SIMD-cycles of the
launch = 1024 SIMDs * GRBM_GUI_ACTIVE / 8 (GRBM_GUI_ACTIVE is summed over the
8 XCDs, MI355X_MICROARCH.md "DVFS"); valu_busy = 2 * SQ_INSTS_VALU / SIMD-cycles,
a LOWER bound on VALU issue occupancy: every wave64 VALU instruction holds its
SIMD >= 2 cycles (add/mul/fma; cvt/floor/cmp/cndmask/min3/med3/u24 take 4,
sqrt/rcp 8: profiles/r01_valu_costs.txt).  (The gfx94x VALUBusy formula,
4 * SQ_ACTIVE_INST_VALU / SIMD-cycles, assumes 4 cycles per instruction and
reads > 1 here; it is kept as valu_busy_gfx94x_formula.)  The clock =
GRBM_GUI_ACTIVE / 8 / kernel duration (reads high below ~0.3 ms).
usage: python tools/prof_summary2.py TAG CONFIG CAMERA FLAGS SAMPLES [SRC]
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

tag, cfg, cam, flags, samples = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
src = sys.argv[6] if len(sys.argv) > 6 else f"gpurun_out/prof_{tag}"
if flags & 0x3000:                                     # glass order / REFLECT_ALL: the general kernels
    ext = 6 if samples > 1 else 5
else:
    ext = 2 if samples > 1 else (1 if flags & 0x30 else 0)
KERNEL = f"k_render<1, false, false, {ext},"          # the bench's timed instantiation (RGBA8, no stats, untiled)
os.makedirs("profiles", exist_ok=True)
shutil.copy(f"{src}/trace/run_kernel_stats.csv", f"profiles/{tag}_kernel_stats.csv")
avg_ns = None
with open(f"{src}/trace/run_kernel_stats.csv") as f:
    for row in csv.DictReader(f):
        if KERNEL in row["Name"]:
            avg_ns = float(row["AverageNs"])
vals = defaultdict(list)
for p in ("fetch", "write", "valu", "tatd"):
    if not os.path.exists(f"{src}/{p}/run_counter_collection.csv"):
        continue
    with open(f"{src}/{p}/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            if KERNEL in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
med = {k: statistics.median(v) for k, v in vals.items()}
fk, wk = med["FETCH_SIZE"], med["WRITE_SIZE"]
raw, corr = (fk + wk) * 1024, (2 * fk + wk) * 1024
clock = med["GRBM_GUI_ACTIVE"] / 8 / avg_ns if avg_ns else None
simd_cycles = 1024 * med["GRBM_GUI_ACTIVE"] / 8
busy = 2 * med["SQ_INSTS_VALU"] / simd_cycles
busy94 = 4 * med["SQ_ACTIVE_INST_VALU"] / simd_cycles
pmc = {"kernel": KERNEL, "config": cfg, "camera": cam, "flags": flags, "samples": samples,
       "launches": {k: len(v) for k, v in vals.items()}, "median_per_launch": med,
       "avg_duration_ns": avg_ns, "hbm_bytes_raw": raw, "hbm_bytes_read_x2": corr,
       "write_bytes": wk * 1024, "valu_busy": busy, "valu_busy_gfx94x_formula": busy94,
       "valu_insts_per_simd_cycle": med["SQ_INSTS_VALU"] / simd_cycles,
       "valu_lane_util": med["SQ_THREAD_CYCLES_VALU"] / (64 * med["SQ_ACTIVE_INST_VALU"]),
       "valu_insts_per_wave": med["SQ_INSTS_VALU"] / med["SQ_WAVES"],
       "issue_stall_share": med["SQ_WAIT_INST_ANY"] / med["SQ_WAVE_CYCLES"],
       "wait_share": med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"],
       "active_share": med["SQ_ACTIVE_INST_ANY"] / med["SQ_WAVE_CYCLES"], "clock_ghz": clock}
if "TA_TA_BUSY_sum" in med:
    # texture address / data units: one of each per CU, shared by its 4 SIMDs (the counters are summed over
    # the 256 CUs; the tatd pass has its own GRBM_GUI_ACTIVE, which the median above mixes: recompute per pass)
    cu_cycles = med["GRBM_GUI_ACTIVE"] / 8
    pmc["ta_busy"] = med["TA_TA_BUSY_sum"] / 256 / cu_cycles
    pmc["td_busy"] = med["TD_TD_BUSY_sum"] / 256 / cu_cycles
    pmc["ta_cycles_per_buffer_load"] = med["TA_TA_BUSY_sum"] / med["TA_BUFFER_READ_WAVEFRONTS_sum"]
json.dump(pmc, open(f"profiles/{tag}_pmc.json", "w"), indent=1)
key = {"config": cfg, "camera": cam, "flags": flags, "samples": samples}
json.dump({**key, "hbm_bytes_per_launch": int(corr), "hbm_bytes_raw": int(raw), "write_bytes": int(wk * 1024),
           "source": f"profiles/{tag}_pmc.json"}, open(f"profiles/traffic_{tag}.json", "w"), indent=1)
json.dump({**key, "valu_busy": round(busy, 4), "valu_lane_util": round(pmc["valu_lane_util"], 4),
           "ta_busy": round(pmc["ta_busy"], 4) if "ta_busy" in pmc else None,
           "td_busy": round(pmc["td_busy"], 4) if "td_busy" in pmc else None,
           "valu_insts_per_wave": round(pmc["valu_insts_per_wave"], 1),
           "issue_stall_share": round(pmc["issue_stall_share"], 4), "wait_share": round(pmc["wait_share"], 4),
           "clock_ghz": round(clock, 3) if clock else None,
           "source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc, tools/profile2.sh)"},
          open(f"profiles/valu_{tag}.json", "w"), indent=1)
print(json.dumps(pmc, indent=1))
