"""Median per-dispatch counter values of the render kernel from tools/pmc.sh output."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

src = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_render<1, false, false,"
vals = defaultdict(list)
for f in sorted(glob.glob(f"{src}/p*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if kern in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
med = {k: statistics.median(v) for k, v in vals.items()}
for k in sorted(med):
    print(f"{k:28s} {med[k]:16.1f}")
def g(k):
    return med.get(k)
if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
    print("VALU lane utilisation      ", g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU")))
if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
    print("VALU insts / wave          ", g("SQ_INSTS_VALU") / g("SQ_WAVES"))
if g("SQ_WAVE_CYCLES") and g("SQ_WAIT_ANY"):
    print("wait share of wave cycles  ", g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"))
    print("issue-stall share          ", g("SQ_WAIT_INST_ANY", ) / g("SQ_WAVE_CYCLES") if g("SQ_WAIT_INST_ANY") else None)
if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
    print("L2 hit rate                ", g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")))
