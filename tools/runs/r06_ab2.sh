#!/bin/bash
# round 6 A/B 2: the primary walk's glass entry and the march loop's tie test as
# wave-uniform branches (pballot, tieb, both) against the head on C3 (full, v1)
# and C5; then C5 block times of the head and of rows rotated to start at 55 %
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
V="head=voxmap_amd/libvoxmap_hip.so pballot=ab/pballot.so tieb=ab/tieb.so both=ab/both.so"
timeout -k 10 300 python -u tools/abtime.py --config C3 --flags 48,0,48,0 --rounds 9 --frames 20 $V > gpurun_out/ab2_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab2_c3.txt; exit 1; }
cat gpurun_out/ab2_c3.txt
timeout -k 10 400 python -u tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 head=voxmap_amd/libvoxmap_hip.so tieb=ab/tieb.so both=ab/both.so > gpurun_out/ab2_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab2_c5.txt; exit 1; }
cat gpurun_out/ab2_c5.txt
for v in btime btime_rot55; do
  timeout -k 10 300 python -u tools/block_times.py ab/$v.so --config C5 --flags 48 --frames 3 --out gpurun_out/block_times_c5_$v.json > gpurun_out/block_times_c5_$v.log 2>&1 || { echo "block times $v failed"; tail -20 gpurun_out/block_times_c5_$v.log; exit 1; }
  tail -3 gpurun_out/block_times_c5_$v.log
done
