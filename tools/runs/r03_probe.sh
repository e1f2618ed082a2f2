#!/bin/bash
# Round-3 probe of what binds the C5 march (run on the GPU box): the TA-rate
# micro-benchmark, then the memory-path PMC passes of tools/profile_mem.sh
# (lat, ta, tcp) for the default soft-shadow path and the pooled one.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
mkdir -p "$ROOT/gpurun_out"
timeout -k 10 120 "$ROOT/tools/micro/ta_rate" > "$ROOT/gpurun_out/ta_rate.txt" 2>&1 || { echo "ta_rate failed"; exit 1; }
cat "$ROOT/gpurun_out/ta_rate.txt"
cd /tmp && export TMPDIR=/tmp
for cfg in "c5def:--config C5 --flags 48" "c5pool:--config C5 --flags 176" "c3:--config C3"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  OUT="$ROOT/gpurun_out/mem_r03_$tag"; mkdir -p "$OUT"
  BASE="$args --no-cpu --no-c5 --inflight 1 --steps 10 --warmup 2 --settle-ms 0"
  for p in "lat:SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "ta:TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
           "tcp:TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
    name=${p%%:*}; ctr=${p#*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$ROOT/bench.py" $BASE > "$OUT/$name.log" 2>&1 || { echo "$tag $name pass failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  done
  echo "done $tag"
done
