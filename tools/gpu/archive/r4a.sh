#!/usr/bin/env bash
# Round 4: the 273-PRB LLR parity diagnostic, then the lower-PHY / chain / HAL GPU tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug/llr_parity_273.py 30 26 > gpurun_out/llr_parity_273.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lower_phy_gpu.py \
  tests/test_chain_gpu.py tests/test_hal_gpu.py > gpurun_out/r4a_tests.log 2>&1
