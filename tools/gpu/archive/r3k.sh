# Round 3: decoder A/B, partner addresses kept (lib, 95 VGPRs, 5 waves / SIMD) vs recomputed (lib_exp_kp0, 79 VGPRs,
# 6 waves / SIMD): headline bench alternated, plus the fixed-iteration Z sweep.
set -o pipefail
mkdir -p gpurun_out/r3k
for i in 1 2; do
  for v in lib lib_exp_kp0; do
    SRSGPU_LIB=$PWD/srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python bench.py --no-extra-workloads --no-extra-points --no-cpu-baseline > gpurun_out/r3k/${v}_$i.json 2> gpurun_out/r3k/${v}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), round(d['roofline']['kernel_ms_per_launch'],4))" gpurun_out/r3k/${v}_$i.json
  done
done
for v in lib lib_exp_kp0; do
  echo $v
  SRSGPU_LIB=$PWD/srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 120 python tools/decoder_scaling.py --z 288 --cols 30 --iters 6 --no-crc --sizes 1024,2048,4096 2>&1 | grep -v amdgpu.ids || exit $?
done
