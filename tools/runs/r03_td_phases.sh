#!/bin/bash
# round 3: TA/TD busy and VALU issue of the C3 render kernel per ablation (which phase loads the texture path)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/td_phases"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for fl in 48 0 8 1 2 4 32; do
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES \
      --kernel-trace --output-format csv -d "$OUT/f$fl" -o run -- python3 "$ROOT/bench.py" --config C3 --flags $fl --no-cpu --no-c5 --no-d2h \
      --inflight 1 --steps 10 --warmup 2 --settle-ms 0 > "$OUT/f$fl.log" 2>&1 || { echo "pass $fl failed"; tail -5 "$OUT/f$fl.log"; exit 1; }
done
echo td phases done
