#!/usr/bin/env bash
# Round 4: upper-PHY slot batches incl. the interpolate time strategy.
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_upper_phy_gpu.py \
  > gpurun_out/r4s_tests.log 2>&1
