#!/bin/bash
# apply tools/ab_patches/brick_late.patch, build with defines=["VX_EXP_BRICK_LATE=8"] into ab/bl8.so, then run this
# round 5: PMC counters of the C5 render launch for the head and the late-brick
# experiment build (ab/bl8.so): VALU / LDS / VMEM instructions and LDS bank
# conflicts (SQ), texture address and data units (TA, TD); one pass each
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/brick_pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--no-cpu --no-c5 --no-d2h --inflight 1 --steps 10 --warmup 2 --settle-ms 0 --config C5"
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TA_BUFFER_READ_WAVEFRONTS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
for v in head:ab/head.so bl8:ab/bl8.so; do
  n=${v%%:*}; lib=$ROOT/${v#*:}
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    VOXMAP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/${n}_p$i" -o run -- \
      python3 "$ROOT/bench.py" $B > "$OUT/${n}_p$i.log" 2>&1 || { echo "$n pass $i failed rc=$?"; tail -5 "$OUT/${n}_p$i.log"; exit 1; }
  done
done
echo brick pmc done
