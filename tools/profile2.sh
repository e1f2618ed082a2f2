#!/bin/bash
# Round-2 rocprofv3 passes for one bench workload (run on the GPU box), each its
# own run under its own time limit, stopping at the first failure:
#   trace  --kernel-trace --stats           per-kernel durations
#   fetch  --pmc FETCH_SIZE                 fabric read bytes per dispatch
#   write  --pmc WRITE_SIZE                 fabric write bytes per dispatch
#   valu   --pmc 8 SQ counters + GRBM_GUI_ACTIVE   VALU issue, waits, clock
#   tatd   --pmc TA/TD busy + buffer wave-loads      the texture address / data path
# usage: TAG=r02 BENCH_ARGS="--config C3" bash tools/profile2.sh
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r02}"
OUT="$ROOT/gpurun_out/prof_$TAG"
BASE="${BENCH_ARGS:-} --no-cpu --no-c5 --no-d2h --inflight 1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" $BASE --steps 100 --warmup 10 > "$OUT/trace.log" 2>&1 || { echo "trace pass failed rc=$?"; tail -5 "$OUT/trace.log"; exit 1; }
P="--steps 10 --warmup 2 --settle-ms 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" $BASE $P > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; tail -5 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" $BASE $P > "$OUT/write.log" 2>&1 || { echo "write pass failed rc=$?"; tail -5 "$OUT/write.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d "$OUT/valu" -o run -- python3 "$ROOT/bench.py" $BASE $P > "$OUT/valu.log" 2>&1 || { echo "valu pass failed rc=$?"; tail -5 "$OUT/valu.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d "$OUT/tatd" -o run -- python3 "$ROOT/bench.py" $BASE $P > "$OUT/tatd.log" 2>&1 || { echo "tatd pass failed rc=$?"; tail -5 "$OUT/tatd.log"; exit 1; }
echo "profile2 passes done ($TAG)"
