# Round 3: decoder traffic / SQ passes for the bench line's secondary workloads (mimo4 at 35 dB, test mode at 30 dB).
set -euo pipefail
EXTRA="--profile mimo4 --snr-db 35" SKIP_BENCH=1 bash tools/gpu_round_profile.sh r3_v1_mimo4
EXTRA="--workload testmode --snr-db 30" SKIP_BENCH=1 bash tools/gpu_round_profile.sh r3_v1_testmode
