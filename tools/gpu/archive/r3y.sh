# Round 3 profile set r3_v2 (fused-dematch decoder, encoder v3): the round profile (default bench, kernel stats, decoder
# FETCH / WRITE / SQ passes) and an SQ pass of the serialised step (every kernel alone: VALU instructions and waits).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
bash tools/gpu_round_profile.sh r3y || exit $?
OUT=gpurun_out/r3y
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d "$R/$OUT/pmc_sq_serial" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-extra-points --no-extra-workloads --steps 40 --warmup 4 --min-time 0 \
  --serial-legs --no-pipeline > "$OUT/pmc_sq_serial.json" 2> "$OUT/pmc_sq_serial.err" || exit $?
SQ_CSV=$(python -c 'import glob, sys; print(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0])' "$OUT/pmc_sq_serial")
python tools/sq_summary.py "$SQ_CSV" "$OUT/sq_serial.json" > "$OUT/sq_serial.log" 2>&1
cat $OUT/sq_serial.log
find "$OUT" -name "*kernel_trace.csv" -delete
find "$OUT" -name "*counter_collection.csv" -size +2M -delete
