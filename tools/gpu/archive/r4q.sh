#!/usr/bin/env bash
# Round 4: kernel trace of the slot-processor benchmark at one thread (the UL slot graph's node timeline).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r4q_prof -o r4q -- python3 -u tools/processor_bench.py \
  --only-slots --threads 1 --repetitions 1 --slots 30 > gpurun_out/r4q_prof.log 2>&1
