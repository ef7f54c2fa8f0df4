#!/usr/bin/env bash
# Round 4: PDSCH modulator chunk size A/B (codeword words per workgroup 256 / 512 / 1024): modulator parity tests per
# build, then the headline bench per build.
set -o pipefail
mkdir -p gpurun_out
for v in lib lib_ab_mod512 lib_ab_mod1024; do
  SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 \
    --timeout-method thread tests/test_pdsch_modulator_gpu.py > gpurun_out/r4h2_tests_$v.log 2>&1 || exit $?
done
for v in lib lib_ab_mod512 lib_ab_mod1024 lib lib_ab_mod512 lib_ab_mod1024; do
  SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python -u bench.py --no-cpu-baseline \
    --no-extra-points --no-extra-workloads >> gpurun_out/r4h2_bench_$v.json 2>> gpurun_out/r4h2_bench.log || exit $?
done
