#!/usr/bin/env bash
# Round 4: lower-PHY processors under a continuous 100 MHz 4-port slot script, reference CPU vs GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lower_phy_bench.py --slots 400 > gpurun_out/r4v_lower_bench.json \
  2> gpurun_out/r4v_lower_bench.log
