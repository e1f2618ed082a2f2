mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L=build/variants
AB_FLAGS="0 48" bash tools/ab.sh prim2:VOXMAP_LIB=$L/prim2.so ms2:VOXMAP_LIB=$L/ms2.so ms1:VOXMAP_LIB=$L/ms1.so prim2:VOXMAP_LIB=$L/prim2.so ms2:VOXMAP_LIB=$L/ms2.so ms1:VOXMAP_LIB=$L/ms1.so || exit 1
AB_FLAGS="48" AB_ARGS="--config C5" bash tools/ab.sh c5ms2:VOXMAP_LIB=$L/ms2.so c5ms1:VOXMAP_LIB=$L/ms1.so
