#!/usr/bin/env bash
# Round 4: slot-processor benchmark, 100 slots per thread and repetition, 1 and 16 threads.
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1
timeout -k 10 400 python -u tools/processor_bench.py --only-slots --threads 16 --repetitions 5 --slots 100 \
  > gpurun_out/r4i_slots_t16.json 2> gpurun_out/r4i_slots_t16.log || exit $?
timeout -k 10 400 python -u tools/processor_bench.py --only-slots --threads 1 --repetitions 3 --slots 100 \
  > gpurun_out/r4i_slots_t1.json 2> gpurun_out/r4i_slots_t1.log
