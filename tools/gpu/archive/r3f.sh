# Round 3: the register-capped decoder build (-DLDPC_PK_MIN_BLOCKS_8=8, srsran-5g_amd/lib_capped) after the scalar
# warm-up fix (ldpc_decoder_common.h: scalar_touch), run once on the decoder tests; then the shipped build's decoder
# tests and the reference processor benchmarks (tools/processor_bench.py).
set -o pipefail
mkdir -p gpurun_out/r3f
SRSGPU_LIB=$PWD/srsran-5g_amd/lib_capped/libsrsgpu_phy.so timeout -k 10 240 python -u -m pytest tests/test_ldpc_decoder_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f/capped_decoder.log 2>&1
rc=$?
tail -4 gpurun_out/r3f/capped_decoder.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u -m pytest tests/test_ldpc_decoder_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f/decoder.log 2>&1
rc=$?
tail -2 gpurun_out/r3f/decoder.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/processor_bench.py > gpurun_out/r3f/processor_bench.json 2> gpurun_out/r3f/processor_bench.err
rc=$?
tail -3 gpurun_out/r3f/processor_bench.err
exit $rc
