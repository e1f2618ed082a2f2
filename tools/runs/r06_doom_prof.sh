#!/bin/bash
# round 6: where the doom table's build goes (k_doom_layer at C5): kernel trace
# and two PMC passes over tools/doom_build_time.py (summaries copied under gpurun_out/)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/doom_prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/tools/doom_build_time.py" > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d "$OUT/sq" -o run -- python3 "$ROOT/tools/doom_build_time.py" > "$OUT/sq.log" 2>&1 || { echo "sq pass failed"; tail -5 "$OUT/sq.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/tools/doom_build_time.py" > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -5 "$OUT/fetch.log"; exit 1; }
cd "$ROOT"
python3 - <<'PY'
import csv, glob, os, statistics, collections
out = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/doom_prof"
for tag in ("sq", "fetch"):
    files = glob.glob(f"{out}/{tag}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if "k_doom_layer" in row.get("Kernel_Name", ""):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(tag, k, "n", len(v), "median", statistics.median(v))
for f in glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "doom" in row["Name"] or "cone" in row["Name"]:
            print("trace", row["Name"][:60], row["Calls"], row["AverageNs"])
PY
rm -rf "$OUT/sq" "$OUT/fetch"
