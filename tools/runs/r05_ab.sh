#!/bin/bash
# round 5: interleaved A/B of library variants (tools/abtime.py); AB_RUNS holds
# one "name|abtime args" per line, variants in AB_LIBS ("label=path ...")
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
while IFS='|' read -r name args; do
  [ -z "$name" ] && continue
  timeout -k 10 600 python tools/abtime.py $args $AB_LIBS > gpurun_out/ab_$name.txt 2>&1 || { echo "ab $name failed rc=$?"; tail gpurun_out/ab_$name.txt; exit 1; }
  cat gpurun_out/ab_$name.txt
done <<< "$AB_RUNS"
