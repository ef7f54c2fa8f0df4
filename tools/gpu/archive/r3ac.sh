# Round 3: full GPU parity suite at the current code, then the stage sensitivity of the headline step.
set -o pipefail
OUT=gpurun_out/r3ac
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for s in none encode dmrs,modulate ofdm_mod ofdm_demod chest demod decode; do
  SRSGPU_BENCH_SKIP=$([ $s = none ] && echo "" || echo $s) timeout -k 10 200 python bench.py $B > $OUT/skip_$s.json 2> $OUT/skip_$s.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step']*1e3,1), 'us/step')" $OUT/skip_$s.json $s
done
