#!/usr/bin/env bash
# Round 4: estimator rework (merged reductions, two DFT stages per barrier, per-symbol rotation table), compact layout
# in the UL slot batch: tests, estimator phase profile, slot benchmark at 16 threads.
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pusch_chest_gpu.py \
  tests/test_ul273_llr_gpu.py tests/test_upper_phy_gpu.py tests/test_chain_gpu.py tests/test_slot_pipeline_gpu.py \
  tests/test_testmode_gpu.py > gpurun_out/r4k_tests.log 2>&1 || exit $?
SRSGPU_LIB=srsran-5g_amd/lib_prof/libsrsgpu_phy.so timeout -k 10 120 python -u tools/chest_phase_profile.py \
  > gpurun_out/r4k_chest_profile.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/processor_bench.py --only-slots --threads 16 --repetitions 5 --slots 100 \
  > gpurun_out/r4k_slots_t16.json 2> gpurun_out/r4k_slots_t16.log
