#!/usr/bin/env bash
# Round 4: demodulator with batched RE loads: parity tests, then the bench's stage times and an SQ pass of the bench.
set -o pipefail
mkdir -p gpurun_out/r4m
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pusch_demodulator_gpu.py \
  tests/test_pusch_chest_gpu.py tests/test_ul273_llr_gpu.py tests/test_slot_pipeline_gpu.py \
  > gpurun_out/r4m/tests.log 2>&1 || exit $?
PB="--no-cpu-baseline --no-extra-points --no-extra-workloads --steps 40 --warmup 4 --min-time 0"
timeout -k 10 300 python bench.py $PB > gpurun_out/r4m/bench.json 2> gpurun_out/r4m/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d "$R/gpurun_out/r4m/pmc_sq" -o run --output-format csv -- \
  python3 "$R/bench.py" $PB > gpurun_out/r4m/pmc_sq.json 2> gpurun_out/r4m/pmc_sq.err || exit $?
SQ_CSV=$(python -c 'import glob, sys; print(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0])' gpurun_out/r4m/pmc_sq)
python tools/sq_summary.py "$SQ_CSV" gpurun_out/r4m/sq_valu.json gpurun_out/r4m/bench.json > gpurun_out/r4m/sq.log 2>&1
find gpurun_out/r4m -name "*counter_collection.csv" -size +2M -delete
