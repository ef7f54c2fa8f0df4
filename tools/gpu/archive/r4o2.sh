#!/usr/bin/env bash
# Round 4: hardware queues at 13 input sets (4 = HIP's default vs 8), headline only, twice each.
set -o pipefail
mkdir -p gpurun_out
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra-points --no-extra-workloads \
    >> gpurun_out/r4o2_q$q.json 2>> gpurun_out/r4o2.log || exit $?
done
