# Round 3: PUSCH channel estimator with two jobs per wave: estimator / receive-chain parity, then headline bench A/B
# against one job per wave (SRSGPU_CHEST_ONE_JOB_PER_WAVE=1).
set -o pipefail
OUT=gpurun_out/r3aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_pusch_chest_gpu.py tests/test_pusch_demodulator_gpu.py tests/test_slot_pipeline_gpu.py tests/test_testmode_gpu.py tests/test_chain_gpu.py tests/test_baseline_configs_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for i in 1 2; do
  for f in 0 1; do
    SRSGPU_CHEST_ONE_JOB_PER_WAVE=$f timeout -k 10 200 python bench.py $B > $OUT/onejob${f}_$i.json 2> $OUT/onejob${f}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), round(d['stage_ms_per_step']['pusch_channel_estimate']*1e3,1), d['pusch_tb_success_rate'], d['ul_llr_parity_vs_reference'] if 'ul_llr_parity_vs_reference' in d else '')" $OUT/onejob${f}_$i.json
  done
done
