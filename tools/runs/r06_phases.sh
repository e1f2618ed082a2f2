#!/bin/bash
# round 6: where the C3 frame goes on the current kernel:
# single-stream phase times by ablation flags (tools/abtime.py, one library) and
# the TA/TD/VALU counters of each ablation (rocprofv3 --pmc, one pass per flag set)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; T=${TAG:-r06}; OUT="$ROOT/gpurun_out/phases_$T"; mkdir -p "$OUT"
FL="48 0 8 1 2 4 16 32"
timeout -k 10 400 python -u tools/abtime.py --config C3 --flags ${FL// /,} --rounds 7 --frames 20 head=voxmap_amd/libvoxmap_hip.so > "$OUT/phase_times.txt" 2>&1 || { echo "abtime failed"; tail -20 "$OUT/phase_times.txt"; exit 1; }
cat "$OUT/phase_times.txt"
cd /tmp && export TMPDIR=/tmp
for fl in $FL; do
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES \
      --kernel-trace --output-format csv -d "$OUT/f$fl" -o run -- python3 "$ROOT/bench.py" --config C3 --flags $fl --no-cpu --no-c5 --no-d2h \
      --inflight 1 --steps 10 --warmup 2 --settle-ms 0 > "$OUT/f$fl.log" 2>&1 || { echo "pass $fl failed"; tail -5 "$OUT/f$fl.log"; exit 1; }
done
cd "$ROOT"
python tools/pmc_ab.py $(for fl in $FL; do echo "$OUT/f$fl"; done) > "$OUT/td_phases_c3.txt"
for fl in $FL; do f=$(ls $OUT/f$fl/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/f$fl/run_kernel_trace.csv); echo "f$fl $(python -c "
import csv,statistics
v=[int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in csv.DictReader(open('$f')) if 'k_render' in r['Kernel_Name']]
print(len(v), statistics.median(v) if v else 0)")"; done >> "$OUT/td_phases_c3.txt"
cat "$OUT/td_phases_c3.txt"
for fl in $FL; do rm -rf "$OUT/f$fl"; done
