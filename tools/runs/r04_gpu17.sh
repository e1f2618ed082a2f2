#!/bin/bash
# round 4: kernel trace of the tile entry box build (k_tile_box + k_render durations)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_tb" -o run -- \
    python3 "$ROOT/bench.py" --config C3 --no-cpu --no-c5 --no-d2h --inflight 1 --steps 50 --warmup 5 > "$ROOT/gpurun_out/prof_tb.log" 2>&1 || { echo "trace failed"; tail -5 "$ROOT/gpurun_out/prof_tb.log"; exit 1; }
cd "$ROOT"; cut -c1-160 gpurun_out/prof_tb/run_kernel_stats.csv | head -12
rm -f gpurun_out/prof_tb/run_kernel_trace.csv
