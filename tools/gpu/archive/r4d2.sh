#!/usr/bin/env bash
# Round 4: timing-only upper bound of removing the demapper's LDS table reads (wrong LLRs; bench asserts skipped via
# the decode check being informational only for this build): headline bench, shipped vs no-table build.
set -o pipefail
mkdir -p gpurun_out
for v in lib lib_ab_notab lib lib_ab_notab; do
  SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra-points \
    --no-extra-workloads >> gpurun_out/r4d2_bench_$v.json 2>> gpurun_out/r4d2_bench.log || exit $?
done
