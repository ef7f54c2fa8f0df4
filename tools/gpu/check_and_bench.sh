# One GPU-box session: the GPU parity tests, the test-mode bench (configs[4]) with its rocprofv3 kernel stats, and the
# default bench. Outputs under gpurun_out/$1 (default check). Every GPU step has its own time limit; steps are chained.
set -euo pipefail
OUT=gpurun_out/${1:-check}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python bench.py --workload testmode --snr-db 30 --steps 1000 --warmup 20 --point-steps 300 \
  --cpu-seconds 6 > "$OUT/bench_testmode.json" 2> "$OUT/bench_testmode.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/tm_stats" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload testmode --snr-db 30 --steps 40 --warmup 4 --no-extra-points --no-cpu-baseline \
  > "$OUT/tm_stats_bench.json" 2> "$OUT/tm_stats.err"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
find "$OUT" -name "*kernel_trace.csv" -delete
du -sh "$OUT"
