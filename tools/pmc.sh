#!/bin/bash
# One rocprofv3 PMC pass per argument (a quoted, space-separated counter set)
# over the bench workload; outputs under gpurun_out/pmc_$TAG/pN/.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-x}"
ARGS="${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu}"
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($set) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo "pmc passes done"
