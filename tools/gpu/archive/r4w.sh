#!/usr/bin/env bash
# Round 4: kernel + copy trace of the lower-PHY bench (PUxCH per-symbol timeline).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r4w_prof -o r4w -- python3 -u \
  tools/lower_phy_bench.py --slots 60 > gpurun_out/r4w.log 2>&1
