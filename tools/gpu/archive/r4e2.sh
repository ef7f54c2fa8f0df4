#!/usr/bin/env bash
# Round 4: codeblock-sharded decode + TB assembly on the device, PUSCH decoder tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_pusch_gpu.py \
  > gpurun_out/r4e2_tests.log 2>&1
