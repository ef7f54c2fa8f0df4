#!/usr/bin/env bash
# Round 4: demodulator lanes chosen per plan: parity tests, then the full bench (headline, operating points, mimo4,
# test mode) with the plan's choice and with 256 lanes forced.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_pusch_demodulator_gpu.py \
  tests/test_pusch_chest_gpu.py tests/test_ul273_llr_gpu.py tests/test_upper_phy_gpu.py tests/test_chain_gpu.py \
  > gpurun_out/r4g2_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r4g2_bench_plan.json 2> gpurun_out/r4g2_bench.log &&
SRSGPU_DEMOD_THREADS=256 timeout -k 10 300 python -u bench.py > gpurun_out/r4g2_bench_256.json 2>> gpurun_out/r4g2_bench.log
