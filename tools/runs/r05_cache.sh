#!/bin/bash
# round 5: L1 (TCP) and L2 (TCC) hit counters of the C3 render launch, full
# quality and primary visibility only (one PMC pass each)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/cache_${TAG:-r05}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CNT="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
B="--no-cpu --no-c5 --no-d2h --inflight 1 --steps 10 --warmup 2 --settle-ms 0 --config C3"
for fl in 48 8; do
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d "$OUT/f$fl" -o run -- \
    python3 "$ROOT/bench.py" $B --flags $fl > "$OUT/f$fl.log" 2>&1 || { echo "pass $fl failed rc=$?"; tail -5 "$OUT/f$fl.log"; exit 1; }
done
echo cache passes done
