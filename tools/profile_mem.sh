#!/bin/bash
# Memory-path PMC passes for one bench workload (run on the GPU box), one
# rocprofv3 run per pass under its own time limit, stopping at the first failure:
#   lat   SQ_INSTS_VMEM_RD, SQ_INST_LEVEL_VMEM, SQ_INSTS_LDS, SQ_INST_LEVEL_LDS,
#         SQ_WAVE_CYCLES, SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE  -> mean vmem latency
#   ta    TA_TA_BUSY_sum, TA_FLAT_READ_WAVEFRONTS_sum, TD_TD_BUSY_sum, TD_SPI_STALL? (skipped)
#   tcp   TCP_TOTAL_CACHE_ACCESSES_sum, TCP_TCC_READ_REQ_sum, TCP_PENDING_STALL_CYCLES_sum, TCP_TCP_TA_DATA_STALL_CYCLES_sum
#   tcc   TCC_HIT_sum, TCC_MISS_sum, TCC_REQ_sum
# usage: TAG=r02_c5 BENCH_ARGS="--config C5" bash tools/profile_mem.sh
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r02}"
OUT="$ROOT/gpurun_out/mem_$TAG"
BASE="${BENCH_ARGS:-} --no-cpu --no-c5 --inflight 1 --steps 10 --warmup 2 --settle-ms 0"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
    name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$ROOT/bench.py" $BASE > "$OUT/$name.log" 2>&1 || { echo "$name pass failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
}
pass lat SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
pass ta TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
echo "profile_mem passes done ($TAG)"
