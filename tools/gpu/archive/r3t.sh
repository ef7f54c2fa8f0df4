# Round 3: rate dematching fused into the packed decoder for plain-copy first transmissions: parity (PUSCH codeblock
# and TB paths, slot pipeline, chain, HAL, baseline configs), then A/B fused vs SRSGPU_DECODER_FUSED_DM=0 on the
# headline bench.
set -o pipefail
mkdir -p gpurun_out/r3t
timeout -k 10 500 python -u -m pytest tests/test_pusch_gpu.py tests/test_ldpc_decoder_gpu.py tests/test_slot_pipeline_gpu.py tests/test_chain_gpu.py tests/test_hal_gpu.py tests/test_baseline_configs_gpu.py tests/test_testmode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3t/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3t/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    SRSGPU_DECODER_FUSED_DM=$f timeout -k 10 200 python bench.py --no-extra-workloads --no-extra-points --no-cpu-baseline > gpurun_out/r3t/fused${f}_$i.json 2> gpurun_out/r3t/fused${f}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), round(d['roofline']['kernel_ms_per_launch'],4), d.get('stages_ms_per_step'))" gpurun_out/r3t/fused${f}_$i.json
  done
done
