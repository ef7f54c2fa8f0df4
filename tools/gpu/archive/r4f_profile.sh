#!/usr/bin/env bash
# Round 4: round profile (bench, kernel stats, decoder traffic, SQ pass) with the final default of 13 input sets.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round_profile.sh r4f
