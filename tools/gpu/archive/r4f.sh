#!/usr/bin/env bash
# Round 4: upper-PHY slot processors with the captured UL slot graph: tests, then the slot benchmark at 1 / 16 threads.
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_upper_phy_gpu.py \
  tests/test_chain_gpu.py > gpurun_out/r4f_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 1 --repetitions 3 --slots 10 \
  > gpurun_out/r4f_slots_t1.json 2> gpurun_out/r4f_slots_t1.log || exit $?
timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 16 --repetitions 3 --slots 10 \
  > gpurun_out/r4f_slots_t16.json 2> gpurun_out/r4f_slots_t16.log
