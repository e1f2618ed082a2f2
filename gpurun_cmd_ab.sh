mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
VOXMAP_LIB=build/variants/pb1024.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu2.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu2.log; [ $rc -eq 0 ] || exit $rc
L=build/variants
AB_FLAGS="0 48" bash tools/ab.sh wg256:VOXMAP_LIB=$L/wg256.so pb:VOXMAP_LIB=$L/pb.so pb1024:VOXMAP_LIB=$L/pb1024.so wg256:VOXMAP_LIB=$L/wg256.so pb:VOXMAP_LIB=$L/pb.so pb1024:VOXMAP_LIB=$L/pb1024.so || exit 1
AB_FLAGS="48" AB_ARGS="--config C5" bash tools/ab.sh c5pb:VOXMAP_LIB=$L/pb.so c5pb1024:VOXMAP_LIB=$L/pb1024.so
