#!/usr/bin/env bash
# Round 4: estimator at 5 vs 6 waves per SIMD (72-78 VGPRs, no spills vs 80 VGPRs, one spill).
set -o pipefail
mkdir -p gpurun_out
SRSGPU_LIB=srsran-5g_amd/lib_ab_p0w5/libsrsgpu_phy.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 \
  --timeout-method thread tests/test_pusch_chest_gpu.py > gpurun_out/r4z2_tests_w5.log 2>&1 || exit $?
for v in lib_ab_p0w5 lib_ab_p0w6 lib_ab_p0w5 lib_ab_p0w6; do
  SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python -u bench.py >> gpurun_out/r4z2_bench_$v.json \
    2>> gpurun_out/r4z2_bench.log || exit $?
done
