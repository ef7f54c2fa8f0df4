#!/usr/bin/env bash
# Round 4: slot-processor benchmark (1 and 16 threads) and a kernel trace of the 1-thread run.
set -o pipefail
mkdir -p gpurun_out
export LIBC_FATAL_STDERR_=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 1 --repetitions 3 --slots 10 \
  > gpurun_out/r4e_slots_t1.json 2> gpurun_out/r4e_slots_t1.log || exit $?
timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 16 --repetitions 3 --slots 10 \
  > gpurun_out/r4e_slots_t16.json 2> gpurun_out/r4e_slots_t16.log || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e_prof -o r4e -- python3 -u tools/processor_bench.py \
  --only-slots --threads 1 --repetitions 1 --slots 10 > gpurun_out/r4e_prof.log 2>&1
