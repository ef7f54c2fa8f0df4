# Round 3: decoder instruction trims (argmin by 32-bit xor, saturating infinity marker): parity, then A/B vs the
# previous arithmetic (lib_exp_old) on the headline bench and the fixed-iteration sweep.
set -o pipefail
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_ldpc_decoder_gpu.py tests/test_pusch_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3s/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3s/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in lib lib_exp_old; do
    SRSGPU_LIB=$PWD/srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python bench.py --no-extra-workloads --no-extra-points --no-cpu-baseline > gpurun_out/r3s/${v}_$i.json 2> gpurun_out/r3s/${v}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), round(d['roofline']['kernel_ms_per_launch'],4))" gpurun_out/r3s/${v}_$i.json
  done
done
for v in lib lib_exp_old; do
  echo $v
  SRSGPU_LIB=$PWD/srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 120 python tools/decoder_scaling.py --z 288 --cols 30 --iters 6 --no-crc --sizes 2048,4096 2>&1 | grep -v amdgpu.ids || exit $?
done
