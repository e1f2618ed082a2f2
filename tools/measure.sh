#!/bin/bash
# Round measurement on the GPU box: headline bench (C3 full quality, CPU
# baseline), C5 bench, then rocprofv3 passes (kernel-trace stats, FETCH_SIZE,
# WRITE_SIZE — each its own run) for both.  Every GPU step has its own time
# limit; the first failure ends the script.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT" || exit 1
mkdir -p gpurun_out
TAG="${TAG:-r01}"
timeout -k 10 300 python bench.py > gpurun_out/bench_c3.log 2>&1 || { echo "bench C3 failed rc=$?"; tail -20 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
timeout -k 10 300 python bench.py --config C5 > gpurun_out/bench_c5.log 2>&1 || { echo "bench C5 failed rc=$?"; tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
# one frame in flight under the profiler: kernel durations not stretched by
# overlap, so rocprofv3's average matches the bench's roofline.avg_launch_ms
TAG=$TAG BENCH_ARGS="--steps 100 --warmup 10 --no-cpu --inflight 1" bash tools/profile.sh || exit 1
TAG=${TAG}_c5 BENCH_ARGS="--config C5 --steps 20 --warmup 3 --no-cpu --inflight 1" bash tools/profile.sh || exit 1
echo "measure done"
