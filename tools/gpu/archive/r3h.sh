# Round 3: decoder throughput vs lifting size at fixed per-lane work (8-layer span, 6 iterations, no CRC): how much a
# partially filled third wave (Z = 288: 144 of 192 lanes) costs against full waves (Z = 256: 128 lanes, Z = 384: 192).
set -o pipefail
mkdir -p gpurun_out/r3h
for z in 256 288 320 352 384; do
  echo "Z=$z"
  timeout -k 10 120 python tools/decoder_scaling.py --z $z --cols 30 --iters 6 --no-crc 2>&1 | grep -v amdgpu.ids || exit $?
done
