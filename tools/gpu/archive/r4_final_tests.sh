#!/usr/bin/env bash
# Round 4: the GPU parity suite and smoke on the final tree (what the driver runs at round end).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/final/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
