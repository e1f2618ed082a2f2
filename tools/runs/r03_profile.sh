#!/bin/bash
# round 3 profiles of the head: C3 (full quality; the same run times v1) and C5,
# each through tools/profile2.sh (kernel trace + FETCH / WRITE / VALU / TA-TD passes)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=r03 BENCH_ARGS="--config C3" bash tools/profile2.sh || exit 1
TAG=r03_c5 BENCH_ARGS="--config C5" bash tools/profile2.sh || exit 1
echo profiles done
