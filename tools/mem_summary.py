"""Per-launch medians of the k_render PMC counters collected by tools/profile_mem.sh
(each counter summed over its instances, per dispatch).
usage: python tools/mem_summary.py gpurun_out/mem_<tag> [...]"""
import collections
import csv
import glob
import statistics
import sys


def summary(d):
    vals = collections.defaultdict(float)
    for f in glob.glob(f"{d}/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "k_render" in r["Kernel_Name"]:
                vals[(f, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (_, _, c), v in vals.items():
        per[c].append(v)
    return {c: statistics.median(v) for c, v in per.items()}


if __name__ == "__main__":
    res = {d: summary(d) for d in sys.argv[1:]}
    names = sorted({c for r in res.values() for c in r})
    print(f"{'counter':36s}" + "".join(f"{d.split('mem_')[-1]:>14s}" for d in res))
    for c in names:
        print(f"{c:36s}" + "".join(f"{r.get(c, float('nan')):14.4g}" for r in res.values()))
    for d, r in res.items():
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in r and "TA_FLAT_READ_WAVEFRONTS_sum" in r:
            print(f"{d}: L1 line accesses per read instruction "
                  f"{r['TCP_TOTAL_CACHE_ACCESSES_sum'] / r['TA_FLAT_READ_WAVEFRONTS_sum']:.1f}, "
                  f"mean vmem latency {r['SQ_INST_LEVEL_VMEM'] / r['SQ_INSTS_VMEM_RD']:.0f} cycles")
