# Round 3 closing set (r3_v3): full GPU parity suite, smoke, the driver-shaped bench, the round profile (default bench,
# kernel stats, decoder FETCH / WRITE / SQ passes) for the headline, mimo4 and test-mode workloads.
set -o pipefail
OUT=gpurun_out/r3ag
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_shape.json 2> $OUT/bench_driver_shape.err || exit $?
bash tools/gpu_round_profile.sh r3ag/headline || exit $?
SKIP_BENCH=1 EXTRA="--profile mimo4 --snr-db 35" bash tools/gpu_round_profile.sh r3ag/mimo4 || exit $?
SKIP_BENCH=1 EXTRA="--workload testmode --snr-db 30" bash tools/gpu_round_profile.sh r3ag/testmode || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), [round(p['value']) for p in d['operating_points']], {k: round(v['value']) for k, v in d.get('workloads', {}).items()})" $OUT/bench_driver_shape.json
