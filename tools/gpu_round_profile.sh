#!/usr/bin/env bash
# One GPU-box session: the default bench (with the CPU reference baseline), a rocprofv3 kernel-trace --stats pass of
# the bench, FETCH_SIZE / WRITE_SIZE PMC passes (separate, per MI355X_MICROARCH.md) for the decoder's HBM traffic and
# an SQ counter pass (VALU issue). Outputs under gpurun_out/$1 (default round). Every GPU step has its own time limit;
# steps are chained (set -e).
set -euo pipefail
OUT=gpurun_out/${1:-round}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
# EXTRA: bench arguments of the profiled workload (e.g. "--profile mimo4 --snr-db 35"); SKIP_BENCH=1: only the passes.
PB="--no-cpu-baseline --no-extra-points --no-extra-workloads --steps 40 --warmup 4 --min-time 0 ${EXTRA:-}"
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/stats" -o run --output-format csv -- \
  python3 "$R/bench.py" $PB > "$OUT/stats_bench.json" 2> "$OUT/stats.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$R/$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" $PB > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$R/$OUT/pmc_write" -o run --output-format csv -- \
  python3 "$R/bench.py" $PB > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d "$R/$OUT/pmc_sq" -o run --output-format csv -- \
  python3 "$R/bench.py" $PB > "$OUT/pmc_sq.json" 2> "$OUT/pmc_sq.err"
python tools/traffic_from_pmc.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/stats_bench.json" "$OUT/traffic.json" \
  > "$OUT/traffic.log" 2>&1
SQ_CSV=$(python -c 'import glob, sys; print(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0])' "$OUT/pmc_sq")
python tools/sq_summary.py "$SQ_CSV" \
  "$OUT/sq_valu.json" "$OUT/stats_bench.json" > "$OUT/sq.log" 2>&1
# Keep the summaries (kernel stats, traffic, SQ) and drop the bulky per-dispatch traces before gpurun copies back.
find "$OUT" -name "*kernel_trace.csv" -delete
find "$OUT" -name "*counter_collection.csv" -size +2M -delete
du -sh "$OUT"
