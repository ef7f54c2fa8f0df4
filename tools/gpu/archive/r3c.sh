# Round-3 binding checks on the GPU box: the HAL thread-pool test, the signal-chain drop-in (reference processors on
# GPU bindings vs CPU) and the test-mode bench at 26 dB with its UL parity check against the reference.
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest tests/test_hal_gpu.py tests/test_chain_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/r3c/hal_chain.log 2>&1
rc=$?
tail -15 gpurun_out/r3c/hal_chain.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --workload testmode --snr-db 26 --no-extra-workloads --no-extra-points --steps 200 --cpu-seconds 4 > gpurun_out/r3c/tm26.json 2> gpurun_out/r3c/tm26.err
tail -c 700 gpurun_out/r3c/tm26.json
