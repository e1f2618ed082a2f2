#!/bin/bash
# End-of-round measurement on the GPU box, every GPU step under its own time
# limit, stopping at the first failure:
#   1. rocprofv3 passes (tools/profile2.sh) for C3 full quality and C5,
#   2. their summaries into profiles/ (bench.py reads traffic_/valu_ files),
#   3. the bench line (C3 headline with v1, C5 and the CPU baseline).
# Everything to keep is copied under gpurun_out/final_<TAG>/.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT" || exit 1
TAG="${TAG:-r02}"
OUT="gpurun_out/final_$TAG"
mkdir -p "$OUT"
TAG=$TAG BENCH_ARGS="--config C3" bash tools/profile2.sh || exit 1
TAG=${TAG}_c5 BENCH_ARGS="--config C5" bash tools/profile2.sh || exit 1
cd "$ROOT" || exit 1
python tools/prof_summary2.py $TAG C3 K1 48 1 > "$OUT/summary_c3.txt" 2>&1 || exit 1
python tools/prof_summary2.py ${TAG}_c5 C5 K1 48 16 > "$OUT/summary_c5.txt" 2>&1 || exit 1
cp profiles/*${TAG}* "$OUT/" || exit 1
timeout -k 10 400 python bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed rc=$?"; tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
echo "final measure done ($TAG)"
