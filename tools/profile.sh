#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box):
#  1. --kernel-trace --stats          per-kernel durations (profiles/*_kernel_stats.csv)
#  2. --pmc FETCH_SIZE  (own pass)     HBM/fabric read bytes per dispatch
#  3. --pmc WRITE_SIZE  (own pass)     write bytes per dispatch
# Each pass under its own timeout; stop at the first failure.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
OUT="$ROOT/gpurun_out/prof_$TAG"
ARGS="${BENCH_ARGS:---steps 20 --warmup 3 --no-cpu}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.log" 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
# byte counters do not depend on the clock: no settle frames under PMC (each dispatch is serialised)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" $ARGS --settle-ms 0 > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" $ARGS --settle-ms 0 > "$OUT/write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "profile passes done"; find "$OUT" -name "*.csv" | head -20
