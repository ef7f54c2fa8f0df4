#!/usr/bin/env bash
# Round 4: the decoder's VALU issue at the worst case (every codeblock runs all 6 iterations) next to the headline:
# stats + SQ passes of the worst-case bench (no FETCH/WRITE passes).
set -o pipefail
OUT=gpurun_out/r4u
mkdir -p $OUT
export TMPDIR=/tmp
R=$(pwd)
PB="--no-cpu-baseline --no-extra-points --no-extra-workloads --steps 40 --warmup 4 --min-time 0 --worst-case"
timeout -k 10 300 python3 bench.py $PB > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d "$R/$OUT/pmc_sq" -o run --output-format csv -- \
  python3 "$R/bench.py" $PB > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || exit $?
SQ_CSV=$(python -c 'import glob, sys; print(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0])' $OUT/pmc_sq)
python tools/sq_summary.py "$SQ_CSV" $OUT/sq_valu.json $OUT/bench.json > $OUT/sq.log 2>&1
find $OUT -name "*counter_collection.csv" -size +2M -delete
