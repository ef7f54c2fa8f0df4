#!/usr/bin/env bash
# Round 4: the upper-PHY slot processors (b6) and the lower-PHY / chain tests, then the estimate-bits diagnostic.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_upper_phy_gpu.py \
  tests/test_lower_phy_gpu.py tests/test_chain_gpu.py tests/test_hal_gpu.py > gpurun_out/r4b_tests.log 2>&1 || exit $?
timeout -k 10 250 python -u tools/debug/chest_bits_273.py > gpurun_out/chest_bits_273.log 2>&1
