# Round 3: decoder FETCH / WRITE / SQ passes for the mimo4 (35 dB) and test-mode (30 dB) workloads at the current code.
set -o pipefail
SKIP_BENCH=1 EXTRA="--profile mimo4 --snr-db 35" bash tools/gpu_round_profile.sh r3z_mimo4 || exit $?
SKIP_BENCH=1 EXTRA="--workload testmode --snr-db 30" bash tools/gpu_round_profile.sh r3z_testmode || exit $?
cat gpurun_out/r3z_mimo4/traffic.json gpurun_out/r3z_testmode/traffic.json
