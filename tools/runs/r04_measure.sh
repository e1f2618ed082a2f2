#!/bin/bash
# round 4 measurements of the head: rocprofv3 passes for C3 and C5
# (tools/profile2.sh), the per-phase PMC ablation of the C3 frame, and the C5
# soft-shadow variants (per-lane march, pooled pass, pooled + LDS bricks) with
# TA/TD and VALU counters
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=r04 BENCH_ARGS="--config C3" bash tools/profile2.sh || exit 1
TAG=r04_c5 BENCH_ARGS="--config C5" bash tools/profile2.sh || exit 1
OUT="$ROOT/gpurun_out/td_phases_r04"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for fl in 48 0 8 1 2 4 32; do
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES \
      --kernel-trace --output-format csv -d "$OUT/f$fl" -o run -- python3 "$ROOT/bench.py" --config C3 --flags $fl --no-cpu --no-c5 --no-d2h \
      --inflight 1 --steps 10 --warmup 2 --settle-ms 0 > "$OUT/f$fl.log" 2>&1 || { echo "pass $fl failed"; tail -5 "$OUT/f$fl.log"; exit 1; }
done
OUT="$ROOT/gpurun_out/c5_soft_r04"; mkdir -p "$OUT"
for fl in 48 176 304; do
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES \
      --kernel-trace --output-format csv -d "$OUT/f$fl" -o run -- python3 "$ROOT/bench.py" --config C5 --flags $fl --no-cpu --no-c5 --no-d2h \
      --inflight 1 --steps 5 --warmup 2 --settle-ms 0 > "$OUT/f$fl.log" 2>&1 || { echo "c5 pass $fl failed"; tail -5 "$OUT/f$fl.log"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
      --kernel-trace --output-format csv -d "$OUT/l$fl" -o run -- python3 "$ROOT/bench.py" --config C5 --flags $fl --no-cpu --no-c5 --no-d2h \
      --inflight 1 --steps 5 --warmup 2 --settle-ms 0 > "$OUT/l$fl.log" 2>&1 || { echo "c5 lds pass $fl failed"; tail -5 "$OUT/l$fl.log"; exit 1; }
done
echo measure passes done
# summaries only (the raw rocprofv3 directories exceed what gpurun copies back)
cd "$ROOT"
python tools/prof_summary2.py r04 C3 K1 48 1 > gpurun_out/summ_r04.log 2>&1 || { echo "summary failed"; tail gpurun_out/summ_r04.log; exit 1; }
python tools/prof_summary2.py r04_c5 C5 K1 48 16 > gpurun_out/summ_r04_c5.log 2>&1 || { echo "summary c5 failed"; tail gpurun_out/summ_r04_c5.log; exit 1; }
mkdir -p gpurun_out/r04_profiles
cp profiles/r04_kernel_stats.csv profiles/r04_pmc.json profiles/traffic_r04.json profiles/valu_r04.json \
   profiles/r04_c5_kernel_stats.csv profiles/r04_c5_pmc.json profiles/traffic_r04_c5.json profiles/valu_r04_c5.json gpurun_out/r04_profiles/
python tools/pmc_ab.py gpurun_out/td_phases_r04/f* > gpurun_out/r04_profiles/td_phases_c3.txt
python tools/pmc_ab.py gpurun_out/c5_soft_r04/* > gpurun_out/r04_profiles/c5_soft.txt
for d in gpurun_out/td_phases_r04 gpurun_out/c5_soft_r04; do for f in $d/*/run_kernel_trace.csv; do echo "$f $(python -c "
import csv,statistics,sys
v=[int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in csv.DictReader(open('$f')) if 'k_render' in r['Kernel_Name']]
print(len(v), statistics.median(v) if v else 0)")"; done; done > gpurun_out/r04_profiles/phase_times.txt
rm -rf gpurun_out/prof_r04 gpurun_out/prof_r04_c5 gpurun_out/td_phases_r04 gpurun_out/c5_soft_r04
echo summaries done
