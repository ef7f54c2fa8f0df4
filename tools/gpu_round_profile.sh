#!/usr/bin/env bash
# One GPU-box session: parity tests, the default bench (with the CPU reference baseline), a rocprofv3 kernel-trace
# --stats pass of the bench, and FETCH_SIZE / WRITE_SIZE PMC passes (separate, per MI355X_MICROARCH.md) for the
# decoder's HBM traffic. Outputs under gpurun_out/round/. Every GPU step has its own time limit; steps are chained.
set -euo pipefail
OUT=gpurun_out/round
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/stats_bench.json" 2> "$OUT/stats.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
python tools/traffic_from_pmc.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/stats_bench.json" "$OUT/traffic.json" \
  > "$OUT/traffic.log" 2>&1
