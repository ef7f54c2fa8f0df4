#!/usr/bin/env bash
# Round 4: step shape at 13 input sets (32 vs 40 vs 48 slots per step), headline only, twice each.
set -o pipefail
mkdir -p gpurun_out
for n in 32 40 48 32 40 48; do
  timeout -k 10 200 python -u bench.py --slots-per-step $n --no-cpu-baseline --no-extra-points --no-extra-workloads \
    >> gpurun_out/r4p2_s$n.json 2>> gpurun_out/r4p2.log || exit $?
done
