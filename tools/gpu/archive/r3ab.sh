# Round 3: decoder A/B, default build (lib) vs lib_exp built with other flags (see the commit using it): decoder parity, then
# (lib_exp built with -DLDPC_PK_PHASED=0): decoder parity, then headline and worst-case bench A/B.
set -o pipefail
OUT=gpurun_out/r3ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ldpc_decoder_gpu.py tests/test_pusch_gpu.py tests/test_hal_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-extra-workloads --no-cpu-baseline --warmup 20 --point-steps 1500"
for i in 1 2; do
  for v in lib lib_exp; do
    SRSGPU_LIB=srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python bench.py $B > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], [round(p['value']) for p in d['operating_points']], round(d['roofline']['kernel_ms_per_launch']*1e3,1))" $OUT/${v}_$i.json
  done
done
