#!/usr/bin/env bash
# Round 4: where the UL slot batch spends a slot at 1 and 16 threads (SRSGPU_BATCH_TIMING phase means).
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1 SRSGPU_BATCH_TIMING=1
timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 1 --repetitions 3 --slots 10 \
  > gpurun_out/r4g_slots_t1.json 2> gpurun_out/r4g_slots_t1.log || exit $?
timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 16 --repetitions 3 --slots 10 \
  > gpurun_out/r4g_slots_t16.json 2> gpurun_out/r4g_slots_t16.log
