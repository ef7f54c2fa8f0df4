#!/usr/bin/env bash
# Round 4: input-set sweep on the final code (headline only): 7 / 9 / 11 / 13 sets, twice each.
set -o pipefail
mkdir -p gpurun_out
for n in 9 7 11 13 9 7 11 13; do
  timeout -k 10 200 python -u bench.py --input-sets $n --no-cpu-baseline --no-extra-points --no-extra-workloads \
    >> gpurun_out/r4l2_sets_$n.json 2>> gpurun_out/r4l2.log || exit $?
done
