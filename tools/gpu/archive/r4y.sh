#!/usr/bin/env bash
# Round 4: slot processors with the DL slot graph (16 and 1 threads).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/processor_bench.py --only-slots --threads 16 --repetitions 5 --slots 100 \
  > gpurun_out/r4y_slots16.json 2> gpurun_out/r4y_slots16.log &&
timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 1 --repetitions 3 --slots 100 \
  > gpurun_out/r4y_slots1.json 2> gpurun_out/r4y_slots1.log
