# Round 3: encoder v2 (Qm = 8 rate matching by bit transposition, core rows over edge chunks, single-wave core parity,
# 8-byte CRC chunks): encoder parity (direct and through the slot / chain / HAL / test-mode paths), phase profile of the
# instrumented build, headline bench.
set -o pipefail
OUT=gpurun_out/r3w
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_pdsch_encoder_gpu.py tests/test_slot_pipeline_gpu.py tests/test_testmode_gpu.py tests/test_hal_gpu.py tests/test_chain_gpu.py tests/test_baseline_configs_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
SRSGPU_LIB=srsran-5g_amd/lib_prof/libsrsgpu_phy.so timeout -k 10 200 python tools/encoder_phase_profile.py --out $OUT/enc_phases.json || exit $?
timeout -k 10 200 python bench.py --no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'], d['stage_ms_per_step'])" $OUT/bench.json
