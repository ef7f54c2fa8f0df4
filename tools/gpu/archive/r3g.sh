# Round 3: A/B of the shipped decoder build (lib) against the register-capped one (lib_capped, 6 waves / SIMD for the
# 8-layer class) on the headline bench, alternated twice; also the worst-case (all iterations) point.
set -o pipefail
mkdir -p gpurun_out/r3g
for i in 1 2; do
  for v in lib lib_capped; do
    SRSGPU_LIB=$PWD/srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python bench.py --no-extra-workloads --no-extra-points --no-cpu-baseline > gpurun_out/r3g/${v}_$i.json 2> gpurun_out/r3g/${v}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['roofline']['achieved'])" gpurun_out/r3g/${v}_$i.json
  done
done
for v in lib lib_capped; do
  SRSGPU_LIB=$PWD/srsran-5g_amd/$v/libsrsgpu_phy.so timeout -k 10 200 python bench.py --worst-case --no-extra-workloads --no-extra-points --no-cpu-baseline > gpurun_out/r3g/${v}_wc.json 2> gpurun_out/r3g/${v}_wc.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'])" gpurun_out/r3g/${v}_wc.json
done
