#!/usr/bin/env bash
# Round 4: estimator waves-per-SIMD A/B: chest parity tests on the shipped build and on each variant, then the headline
# bench per variant.
set -o pipefail
mkdir -p gpurun_out
t() { timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_pusch_chest_gpu.py "$@"; }
t > gpurun_out/r4z_tests_base.log 2>&1 || exit $?
SRSGPU_LIB=srsran-5g_amd/lib_ab_p0w7/libsrsgpu_phy.so t > gpurun_out/r4z_tests_w7.log 2>&1 || exit $?
SRSGPU_LIB=srsran-5g_amd/lib_ab_p0w6/libsrsgpu_phy.so t > gpurun_out/r4z_tests_w6.log 2>&1 || exit $?
for v in lib lib_ab_p0w7 lib_ab_p0w6 lib lib_ab_p0w7 lib_ab_p0w6; do
  SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python -u bench.py >> gpurun_out/r4z_bench_$v.json \
    2>> gpurun_out/r4z_bench.log || exit $?
done
