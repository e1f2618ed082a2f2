#!/bin/bash
# round 4: instruction / wait counters of the C3 v1 render, quad split (flags 0)
# against the unit split (2048) and full quality (48 / 2096), same library
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_quad"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P="--config C3 --no-cpu --no-c5 --no-d2h --inflight 1 --steps 10 --warmup 2 --settle-ms 0"
for fl in 0 2048 48 2096; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d "$OUT/f$fl" -o run -- python3 "$ROOT/bench.py" $P --flags $fl > "$OUT/f$fl.log" 2>&1 || { echo "pass $fl failed rc=$?"; tail -5 "$OUT/f$fl.log"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d "$OUT/t$fl" -o run -- python3 "$ROOT/bench.py" $P --flags $fl > "$OUT/t$fl.log" 2>&1 || { echo "pass t$fl failed rc=$?"; tail -5 "$OUT/t$fl.log"; exit 1; }
done
cd "$ROOT" && python tools/pmc_ab.py "$OUT"/f0 "$OUT"/f2048 "$OUT"/f48 "$OUT"/f2096 "$OUT"/t0 "$OUT"/t2048 "$OUT"/t48 "$OUT"/t2096 | tee gpurun_out/pmc_quad.txt
