# Round 3 closing set with the new step structure (DL / UL leg graphs, 9 input sets; r3_v4): smoke, the default bench
# (wall time recorded), the driver-shaped bench, and the round profile of the headline.
set -o pipefail
OUT=gpurun_out/r3aj
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
s0=$(date +%s); timeout -k 10 500 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
echo "default bench wall s: $(( $(date +%s) - s0 ))"
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_shape.json 2> $OUT/bench_driver_shape.err || exit $?
for f in bench_default bench_driver_shape; do
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), d['steps'], [round(p['value']) for p in d['operating_points']], {k: round(v['value']) for k, v in d.get('workloads', {}).items()}, (d['cpu_baseline'] or {}).get('value'))" $OUT/$f.json
done
SKIP_BENCH=1 bash tools/gpu_round_profile.sh r3aj/headline || exit $?
