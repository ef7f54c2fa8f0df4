#!/usr/bin/env bash
# Round 4: sliced TB stage for large segmented TBs: decoder / chain / slot-processor / test-mode tests, the full bench
# (test mode decodes 37 KB TBs), then the slot-processor benchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pusch_gpu.py \
  tests/test_upper_phy_gpu.py tests/test_chain_gpu.py tests/test_hal_gpu.py tests/test_testmode_gpu.py \
  tests/test_ul273_llr_gpu.py > gpurun_out/r4j2_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4j2_bench.json 2> gpurun_out/r4j2_bench.log &&
timeout -k 10 400 python -u tools/processor_bench.py --only-slots --threads 16 --repetitions 5 --slots 100 \
  > gpurun_out/r4j2_slots16.json 2> gpurun_out/r4j2_slots16.log &&
timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 1 --repetitions 3 --slots 100 \
  > gpurun_out/r4j2_slots1.json 2> gpurun_out/r4j2_slots1.log
