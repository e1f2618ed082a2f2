#!/bin/bash
# round 4: the default bench line (N = 1) on the head
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r04.jsonl 2> gpurun_out/bench_r04.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_r04.err; exit 1; }
tail -c 3000 gpurun_out/bench_r04.jsonl
