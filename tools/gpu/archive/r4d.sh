#!/usr/bin/env bash
# Round 4: the upper-PHY slot processors (b6), lower-PHY / chain / HAL tests, then the slot-processor benchmark.
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_upper_phy_gpu.py \
  tests/test_lower_phy_gpu.py tests/test_chain_gpu.py tests/test_hal_gpu.py > gpurun_out/r4d_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/processor_bench.py --only-slots --repetitions 3 --slots 10 \
  > gpurun_out/r4d_processor_bench.log 2>&1
