"""Per-launch medians of every counter of the bench's render kernel in a
rocprofv3 --pmc output directory: python tools/pmc_ab.py DIR [DIR ...]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    vals = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "k_render" not in row["Kernel_Name"]:
                    continue
                vals[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    med = {k: statistics.median(v.values()) for k, v in vals.items()}
    print(d, " ".join(f"{k}={v:.4g}" for k, v in sorted(med.items())), flush=True)
