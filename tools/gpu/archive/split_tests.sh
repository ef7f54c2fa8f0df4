# Decoder parity with the edge-split kernel forced, then the default selection, then a bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SRSGPU_DECODER_SPLIT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ldpc or pusch or hal or smoke or slot or baseline" > gpurun_out/split_tests.log 2>&1 || { tail -30 gpurun_out/split_tests.log; exit 1; }
tail -2 gpurun_out/split_tests.log
bash tools/gpu/bench_ab.sh "" "--input-sets 8" || exit 1
SRSGPU_DECODER_SPLIT=0 bash tools/gpu/bench_ab.sh ""
