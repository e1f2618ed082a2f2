mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L=build/variants
AB_FLAGS="0 48" bash tools/ab.sh base:VOXMAP_LIB=$L/base.so rcp:VOXMAP_LIB=$L/rcp.so base:VOXMAP_LIB=$L/base.so rcp:VOXMAP_LIB=$L/rcp.so base:VOXMAP_LIB=$L/base.so rcp:VOXMAP_LIB=$L/rcp.so
