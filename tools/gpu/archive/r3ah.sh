# Round 3: encoder 256QAM groups written as two 16-byte stores: encoder parity, then two headline bench runs (compare
# with profiles/r3_v3_bench*.json, 129.9k-130.0k on an earlier box).
set -o pipefail
OUT=gpurun_out/r3ah
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_pdsch_encoder_gpu.py tests/test_slot_pipeline_gpu.py tests/test_testmode_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for i in 1 2; do
  timeout -k 10 200 python bench.py $B > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[1], round(d['value']), round(s['pdsch_encode']*1e3,1))" $OUT/bench_$i.json
done
