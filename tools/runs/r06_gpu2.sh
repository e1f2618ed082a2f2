#!/bin/bash
# round 6: the new list / cone GPU tests, the whole GPU suite, smoke, the glass-lattice stress timing
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lists_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/lists_r06.log 2>&1 || { echo "list tests failed rc=$?"; tail -30 gpurun_out/lists_r06.log; exit 1; }
tail -2 gpurun_out/lists_r06.log
TAG=r06b bash tools/runs/r06_gpu_tests.sh || exit 1
timeout -k 10 400 python -u tools/glass_lattice.py --out gpurun_out/glass_lattice_r06.json > gpurun_out/glass_lattice_r06.log 2>&1 || { echo "lattice failed rc=$?"; tail -20 gpurun_out/glass_lattice_r06.log; exit 1; }
cat gpurun_out/glass_lattice_r06.log
