#!/usr/bin/env bash
# Round 4: OFDM kernels forced to 5 waves per SIMD (96 VGPRs, 12-25 spilled) vs the shipped build (4 waves, no spill):
# OFDM parity tests on the variant, then the headline bench per build.
set -o pipefail
mkdir -p gpurun_out
SRSGPU_LIB=srsran-5g_amd/lib_ab_ofdm5/libsrsgpu_phy.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 \
  --timeout-method thread tests/test_ofdm_gpu.py > gpurun_out/r4q2_tests.log 2>&1 || exit $?
for v in lib lib_ab_ofdm5 lib lib_ab_ofdm5; do
  SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python -u bench.py --no-cpu-baseline \
    --no-extra-points --no-extra-workloads >> gpurun_out/r4q2_bench_$v.json 2>> gpurun_out/r4q2_bench.log || exit $?
done
