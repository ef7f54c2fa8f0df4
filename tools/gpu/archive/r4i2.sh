#!/usr/bin/env bash
# Round 4: PDSCH modulator chunk / workgroup A/B, second pass: 1024 words x 256 lanes vs 1024 x 128 vs 2048 x 256.
set -o pipefail
mkdir -p gpurun_out
for v in lib_ab_mod1024_128 lib_ab_mod2048_256; do
  SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 \
    --timeout-method thread tests/test_pdsch_modulator_gpu.py tests/test_pusch_demodulator_gpu.py \
    > gpurun_out/r4i2_tests_$v.log 2>&1 || exit $?
done
for v in lib_ab_mod1024 lib_ab_mod1024_128 lib_ab_mod2048_256 lib_ab_mod1024 lib_ab_mod1024_128 lib_ab_mod2048_256; do
  SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python -u bench.py --no-cpu-baseline \
    --no-extra-points --no-extra-workloads >> gpurun_out/r4i2_bench_$v.json 2>> gpurun_out/r4i2_bench.log || exit $?
done
