set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r5g_trace
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/$OUT/kt" -o run --output-format csv -- python3 "$PWD/bench.py" --no-cpu-baseline --no-extra-points --no-extra-workloads --steps 300 --warmup 20 --min-time 0 > $OUT/bench.json 2> $OUT/bench.err
f=$(find $OUT/kt -name "*kernel_trace.csv" | head -1); gzip -c "$f" > $OUT/kernel_trace.csv.gz; find $OUT/kt -name "*kernel_trace.csv" -delete; ls -la $OUT
