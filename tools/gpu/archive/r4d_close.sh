#!/usr/bin/env bash
# Round 4 closing set r4d (after the demodulator lanes and modulator chunks): the GPU parity suite, smoke, then the round profile (bench, kernel stats, decoder traffic,
# SQ pass) of the headline workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4d
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4d/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4d/smoke.log 2>&1 || exit $?
bash tools/gpu_round_profile.sh r4d
