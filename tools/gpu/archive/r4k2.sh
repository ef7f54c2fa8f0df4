#!/usr/bin/env bash
# Round 4: sliced TB stage A/B on the test-mode workload (37 KB TBs) and the one-PDU UL slot processor.
set -o pipefail
mkdir -p gpurun_out
for v in 1 0 1 0; do
  SRSGPU_TB_SLICED=$v timeout -k 10 200 python -u bench.py --workload testmode --snr-db 30 --no-cpu-baseline \
    --no-extra-points --no-extra-workloads >> gpurun_out/r4k2_testmode_$v.json 2>> gpurun_out/r4k2.log || exit $?
done
for v in 1 0; do
  SRSGPU_TB_SLICED=$v timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 1 --repetitions 3 \
    --slots 100 > gpurun_out/r4k2_slots1_$v.json 2>> gpurun_out/r4k2.log || exit $?
done
