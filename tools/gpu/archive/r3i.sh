# Round 3: the multi-codeblock decoder (PK4): decoder parity for every kernel variant, then the lifting-size sweep and
# the headline bench A/B (PK4 off / on).
set -o pipefail
mkdir -p gpurun_out/r3i
timeout -k 10 300 python -u -m pytest tests/test_ldpc_decoder_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i/decoder.log 2>&1
rc=$?; tail -5 gpurun_out/r3i/decoder.log; [ $rc -eq 0 ] || exit $rc
for z in 288 352; do
  for v in 0 1; do
    echo "Z=$z PK4=$v"
    SRSGPU_DECODER_PK4=$v timeout -k 10 120 python tools/decoder_scaling.py --z $z --cols 30 --iters 6 --no-crc 2>&1 | grep -v amdgpu.ids || exit $?
  done
done > gpurun_out/r3i/scaling.log
cat gpurun_out/r3i/scaling.log
for i in 1 2; do
  for v in 0 1; do
    SRSGPU_DECODER_PK4=$v timeout -k 10 200 python bench.py --no-extra-workloads --no-extra-points --no-cpu-baseline > gpurun_out/r3i/bench_pk4_${v}_$i.json 2> gpurun_out/r3i/bench_pk4_${v}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['roofline']['achieved'], d.get('roofline_valu',{}).get('frac'))" gpurun_out/r3i/bench_pk4_${v}_$i.json
  done
done
