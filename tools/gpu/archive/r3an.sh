# Round 3: kernel overlap of the leg-graph step structure (rocprofv3 --kernel-trace of 300 timed steps).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=gpurun_out/r3an
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$OUT/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-extra-points --no-extra-workloads --steps 300 --warmup 20 --min-time 0 \
  > $OUT/bench.json 2> $OUT/bench.err || exit $?
CSV=$(python -c 'import glob, sys; print(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])' "$OUT/trace")
python tools/overlap_from_trace.py "$CSV" $OUT/overlap.json > $OUT/overlap.log 2>&1 || exit $?
head -c 600 $OUT/overlap.json
find "$OUT" -name "*kernel_trace.csv" -delete
