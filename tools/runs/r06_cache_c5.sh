#!/bin/bash
# round 6: L1 (TCP) and L2 (TCC) hit counters of the C5 render launch (one PMC pass)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/cache_c5_${TAG:-r06}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CNT="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
B="--no-cpu --no-c5 --no-d2h --inflight 1 --steps 5 --warmup 2 --settle-ms 0 --config C5"
timeout -s KILL 150 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d "$OUT/c5" -o run -- \
    python3 "$ROOT/bench.py" $B > "$OUT/c5.log" 2>&1 || { echo "pass failed rc=$?"; tail -5 "$OUT/c5.log"; exit 1; }
cd "$ROOT" && python tools/pmc_ab.py "$OUT/c5"
