#!/bin/bash
# round 3: every GPU test, then a short bench line without the CPU baseline
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | grep -E "exit_gpu|FAILED|ERROR" | head -20; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --steps 50 > gpurun_out/bench_quick.jsonl 2> gpurun_out/bench_quick.err || { echo "bench failed"; tail gpurun_out/bench_quick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_quick.jsonl')); print(d['value'], d['config']['exit_tables'], d['config']['c5']['exit_tables'])"
