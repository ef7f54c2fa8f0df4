# Round 3: PUSCH demodulator descriptor loaded in parallel with the chunk (one chunk per transmission; default) vs
# through the chunk's index (SRSGPU_DEMOD_DIRECT=0): demodulator / receive-chain parity, then the headline bench A/B.
set -o pipefail
OUT=gpurun_out/r3af
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_pusch_demodulator_gpu.py tests/test_pusch_chest_gpu.py tests/test_slot_pipeline_gpu.py tests/test_chain_gpu.py tests/test_ulsch_demux_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for i in 1 2; do
  for f in 1 0; do
    SRSGPU_DEMOD_DIRECT=$f timeout -k 10 200 python bench.py $B > $OUT/direct${f}_$i.json 2> $OUT/direct${f}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[1], round(d['value']), round(s['pusch_demodulate']*1e3,1))" $OUT/direct${f}_$i.json
  done
done
