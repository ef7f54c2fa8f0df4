# Round 3: PK4 decoder with 8-wave workgroups (two per CU at 5 waves / SIMD) vs the one-codeblock kernel: fixed
# 6-iteration Z sweep and the headline bench.
set -o pipefail
mkdir -p gpurun_out/r3o
for cfg in "0 0" "1 512" "1 0"; do
  set -- $cfg
  echo "PK4=$1 THREADS=$2"
  for z in 288 352; do
    SRSGPU_DECODER_PK4=$1 SRSGPU_DECODER_PK4_THREADS=$2 timeout -k 10 120 python tools/decoder_scaling.py --z $z --cols 30 --iters 6 --no-crc --sizes 2048,4096 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
for cfg in "0 0" "1 512"; do
  set -- $cfg
  SRSGPU_DECODER_PK4=$1 SRSGPU_DECODER_PK4_THREADS=$2 timeout -k 10 200 python bench.py --no-extra-workloads --no-extra-points --no-cpu-baseline > gpurun_out/r3o/bench_$1_$2.json 2> gpurun_out/r3o/bench_$1_$2.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), round(d['roofline']['kernel_ms_per_launch'],4))" gpurun_out/r3o/bench_$1_$2.json
done
