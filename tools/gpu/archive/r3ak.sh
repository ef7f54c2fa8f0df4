# Round 3: driver-shaped bench after the every-set warm-up fix (9 input sets, --warmup 5).
set -o pipefail
OUT=gpurun_out/r3ak
mkdir -p $OUT
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_shape.json 2> $OUT/bench_driver_shape.err || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), d['steps'], [round(p['value']) for p in d['operating_points']], {k: round(v['value']) for k, v in d.get('workloads', {}).items()}, (d['cpu_baseline'] or {}).get('value'))" $OUT/bench_driver_shape.json
