#!/usr/bin/env bash
# Round 4: PUSCH demodulator lanes per chunk A/B (SRSGPU_DEMOD_THREADS 256 / 128 / 64): demodulator parity tests at
# each size, then the headline bench per size.
set -o pipefail
mkdir -p gpurun_out
for t in 256 128 64; do
  SRSGPU_DEMOD_THREADS=$t timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
    tests/test_pusch_demodulator_gpu.py > gpurun_out/r4f2_tests_$t.log 2>&1 || exit $?
done
for t in 256 128 64 256 128 64; do
  SRSGPU_DEMOD_THREADS=$t timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra-points \
    --no-extra-workloads >> gpurun_out/r4f2_bench_$t.json 2>> gpurun_out/r4f2_bench.log || exit $?
done
