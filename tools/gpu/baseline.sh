set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2a/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2a/bench_prof.json 2>&1
