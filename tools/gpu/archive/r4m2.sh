#!/usr/bin/env bash
# Round 4: input-set sweep on the final code (headline only): 13 / 16 / 20 / 24 sets, twice each.
set -o pipefail
mkdir -p gpurun_out
for n in 16 20 24 13 16 20 24 13; do
  timeout -k 10 200 python -u bench.py --input-sets $n --no-cpu-baseline --no-extra-points --no-extra-workloads \
    >> gpurun_out/r4m2_sets_$n.json 2>> gpurun_out/r4m2.log || exit $?
done
