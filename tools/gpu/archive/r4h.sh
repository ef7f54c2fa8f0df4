#!/usr/bin/env bash
# Round 4: the slot benchmark at 16 threads with 8 and 16 hardware queues per process (HIP's default is 4).
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 16 --repetitions 3 \
    --slots 10 > gpurun_out/r4h_slots_t16_q$q.json 2> gpurun_out/r4h_slots_t16_q$q.log || exit $?
done
