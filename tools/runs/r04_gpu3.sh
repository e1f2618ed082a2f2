#!/bin/bash
# round 4: the head against the round-3 head (ab/lib_r03.so, git 69ca0cd) and the
# previous head (ab/lib_qspec.so) in one process; per-block times of one launch
# (ab/lib_btime.so, -DVX_BLOCK_TIMING); the golden / parity GPU tests.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python tools/abtime.py --config C3 --flags 48,0 --rounds 7 new=voxmap_amd/libvoxmap_hip.so qspec=ab/lib_qspec.so r03=ab/lib_r03.so > gpurun_out/ab_r03_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_r03_c3.txt; exit 1; }
cat gpurun_out/ab_r03_c3.txt
timeout -k 10 400 python tools/abtime.py --config C5 --flags 48 --rounds 3 --frames 10 new=voxmap_amd/libvoxmap_hip.so r03=ab/lib_r03.so > gpurun_out/ab_r03_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_r03_c5.txt; exit 1; }
cat gpurun_out/ab_r03_c5.txt
timeout -k 10 200 python tools/block_times.py ab/lib_btime.so --config C5 --out gpurun_out/btime_c5.json > gpurun_out/btime_c5.log 2>&1 || { echo "btime c5 failed"; tail gpurun_out/btime_c5.log; exit 1; }
timeout -k 10 200 python tools/block_times.py ab/lib_btime.so --config C3 --out gpurun_out/btime_c3.json > gpurun_out/btime_c3.log 2>&1 || { echo "btime c3 failed"; tail gpurun_out/btime_c3.log; exit 1; }
python -c "
import json
for c in ('c5','c3'):
    d=json.load(open('gpurun_out/btime_%s.json'%c))
    for f in d['frames'][:2]: print(c, {k:v for k,v in f.items() if k!='row_mean_us'})
"
timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_par.log; exit $rc
