#!/usr/bin/env bash
# Round 4: estimator phase profile incl. the bench's slot shape (instrumented build).
set -o pipefail
mkdir -p gpurun_out
SRSGPU_LIB=srsran-5g_amd/lib_prof/libsrsgpu_phy.so timeout -k 10 120 python -u tools/chest_phase_profile.py \
  > gpurun_out/r4r_chest_profile.log 2>&1
