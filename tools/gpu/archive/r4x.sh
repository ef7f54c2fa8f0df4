#!/usr/bin/env bash
# Round 4: PUxCH per-symbol graphs: lower-PHY and upper-PHY tests, then the lower-PHY bench.
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lower_phy_gpu.py \
  tests/test_upper_phy_gpu.py tests/test_chain_gpu.py tests/test_hal_gpu.py > gpurun_out/r4x_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/lower_phy_bench.py --slots 400 > gpurun_out/r4x_lower_bench.json \
  2> gpurun_out/r4x_lower_bench.log
