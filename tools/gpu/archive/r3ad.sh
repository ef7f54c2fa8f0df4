# Round 3: OFDM two symbols per workgroup (power-of-two sizes from 1024 points): OFDM / slot / chain parity, then the
# headline bench A/B against one symbol per workgroup (SRSGPU_OFDM_ONE_SYMBOL=1).
set -o pipefail
OUT=gpurun_out/r3ad
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ofdm_gpu.py tests/test_slot_pipeline_gpu.py tests/test_testmode_gpu.py tests/test_chain_gpu.py tests/test_baseline_configs_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for i in 1 2; do
  for f in 0 1; do
    SRSGPU_OFDM_ONE_SYMBOL=$f timeout -k 10 200 python bench.py $B > $OUT/one${f}_$i.json 2> $OUT/one${f}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[1], round(d['value']), round(s['ofdm_modulate']*1e3,1), round(s['ofdm_demodulate']*1e3,1), d['pusch_tb_success_rate'])" $OUT/one${f}_$i.json
  done
done
