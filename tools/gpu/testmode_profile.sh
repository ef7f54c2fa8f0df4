# Test-mode (configs[4]) bench and its rocprofv3 kernel stats under gpurun_out/$1 (default testmode).
set -euo pipefail
OUT=gpurun_out/${1:-testmode}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python bench.py --workload testmode --snr-db 30 --point-steps 1000 --cpu-seconds 8 \
  > "$OUT/bench_testmode.json" 2> "$OUT/bench_testmode.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/tm_stats" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload testmode --snr-db 30 --steps 40 --warmup 4 --no-extra-points --no-cpu-baseline \
  > "$OUT/tm_stats_bench.json" 2> "$OUT/tm_stats.err"
find "$OUT" -name "*kernel_trace.csv" -delete
