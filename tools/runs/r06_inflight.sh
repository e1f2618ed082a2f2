#!/bin/bash
# round 6: frames in flight (streams) 4 / 6 / 8 on the C3 full-quality line
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
for k in 4 8 6 4 8; do
  timeout -k 10 200 python -u bench.py --inflight $k --no-cpu --no-c5 --no-d2h --steps 100 --warmup 10 > gpurun_out/inflight_$k.jsonl 2> gpurun_out/inflight_$k.err || { echo "bench k=$k failed"; tail -5 gpurun_out/inflight_$k.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/inflight_$k.jsonl').read().strip().splitlines()[-1]); print('inflight $k', d['value'], d['ms_per_step'], d['config']['inflight'])"
done
