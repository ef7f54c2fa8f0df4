# Round 3: PUSCH demodulator at 6 waves per SIMD (lib_exp: -DSRSGPU_DEMOD_WAVES=6, 80 VGPRs, 1 spilled) vs the
# default 5 (92 VGPRs): demodulator parity on the variant, then the headline bench A/B.
set -o pipefail
OUT=gpurun_out/r3ae
mkdir -p $OUT
SRSGPU_LIB=srsran-5g_amd/lib_exp/libsrsgpu_phy.so timeout -k 10 600 python -u -m pytest tests/test_pusch_demodulator_gpu.py tests/test_slot_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for i in 1 2; do
  for v in lib lib_exp; do
    SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python bench.py $B > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[1], round(d['value']), round(s['pusch_demodulate']*1e3,1))" $OUT/${v}_$i.json
  done
done
