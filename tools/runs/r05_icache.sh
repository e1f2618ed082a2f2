#!/bin/bash
# round 5: instruction-cache counters on the C3 and C5 render launches (one PMC pass each)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/icache_${TAG:-r05}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || { echo "list-avail failed"; exit 1; }
grep -E "^ *(SQC_ICACHE|SQ_IFETCH|SQ_INST_LEVEL|SQC_TC_INST|SQ_WAIT_INST)" "$OUT/avail.txt" | head -40 || true
grep -o -E "SQC_ICACHE[A-Z_]*|SQ_IFETCH[A-Z_]*|SQ_WAIT_INST[A-Z_]*" "$OUT/avail.txt" | sort -u
CNT="${CNT:-SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE}"
for c in $CNT; do grep -q -w "$c" "$OUT/avail.txt" || { echo "counter $c not listed"; exit 1; }; done
B="--no-cpu --no-c5 --no-d2h --inflight 1 --steps 10 --warmup 2 --settle-ms 0"
for cfg in C3 C5; do
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d "$OUT/$cfg" -o run -- \
    python3 "$ROOT/bench.py" $B --config $cfg > "$OUT/$cfg.log" 2>&1 || { echo "$cfg pass failed rc=$?"; tail -5 "$OUT/$cfg.log"; exit 1; }
done
echo icache passes done
