#!/usr/bin/env bash
# Round 4: estimator DPP reductions (chest parity), upper-PHY slot processors (b6), lower-PHY / chain tests, then the
# estimate-bits diagnostic.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_pusch_chest_gpu.py tests/test_pusch_demodulator_gpu.py tests/test_ul273_llr_gpu.py -s \
  tests/test_pusch_gpu.py > gpurun_out/r4c_chest.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_upper_phy_gpu.py \
  tests/test_lower_phy_gpu.py tests/test_chain_gpu.py tests/test_hal_gpu.py > gpurun_out/r4c_tests.log 2>&1 || exit $?
timeout -k 10 250 python -u tools/debug/chest_bits_273.py > gpurun_out/chest_bits_273.log 2>&1
