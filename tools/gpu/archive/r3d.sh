# Full GPU parity suite (one pytest process), then the default bench (driver command shape).
mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3d/gpu_tests.log 2>&1
rc=$?
tail -12 gpurun_out/r3d/gpu_tests.log
exit $rc
