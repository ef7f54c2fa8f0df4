# Round 3: OFDM parity incl. the split-transform sizes (9216 .. 98304), then the decoder issue-breakdown PMC passes.
set -o pipefail
mkdir -p gpurun_out/r3n
timeout -k 10 300 python -u -m pytest tests/test_ofdm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n/ofdm.log 2>&1
rc=$?; tail -4 gpurun_out/r3n/ofdm.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r3m.sh
