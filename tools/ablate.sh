#!/bin/bash
# Frame time with parts of the shading switched off (VX_FLAG_* bits), one process each.
# 0 = v1, 1 no shadow, 2 no AO, 4 no clouds, 8 primary only, 16 reflect, 32 rough, 48 full quality.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in ${ABL_FLAGS:-0 1 2 4 8 16 32 48 49 50}; do
  timeout -k 10 120 python bench.py --no-cpu --steps 30 --warmup 3 --flags $f ${ABL_ARGS} > gpurun_out/ablate_$f.log 2>&1 || exit $?
  echo "flags=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ablate_$f.log)"
done
