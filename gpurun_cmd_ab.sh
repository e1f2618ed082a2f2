mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L=build/variants
AB_FLAGS="48" AB_ARGS="--config C5 --samples 16" bash tools/ab.sh c5m0b0:VOXMAP_LIB=$L/m0b0.so c5rot0:VOXMAP_LIB=$L/rot_b0.so c5rot1:VOXMAP_LIB=$L/rot_b1.so || exit 1
AB_FLAGS="0 48" bash tools/ab.sh m0b0:VOXMAP_LIB=$L/m0b0.so rot0:VOXMAP_LIB=$L/rot_b0.so rot1:VOXMAP_LIB=$L/rot_b1.so m0b0:VOXMAP_LIB=$L/m0b0.so rot0:VOXMAP_LIB=$L/rot_b0.so rot1:VOXMAP_LIB=$L/rot_b1.so
