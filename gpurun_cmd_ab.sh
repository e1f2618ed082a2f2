mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "field_build or from_grid" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b3.log 2>&1 || { tail -20 gpurun_out/b3.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"scene_build_s": [0-9.]*' gpurun_out/b3.log
timeout -k 10 300 python bench.py --no-cpu --config C5 > gpurun_out/b5.log 2>&1 || { tail -20 gpurun_out/b5.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"scene_build_s": [0-9.]*' gpurun_out/b5.log
