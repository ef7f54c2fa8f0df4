#!/usr/bin/env bash
# Round 4: the default bench (13 input sets) and the driver's shape on the final code.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r4n2_bench.json 2> gpurun_out/r4n2_bench.log &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4n2_bench_driver.json 2>> gpurun_out/r4n2_bench.log
