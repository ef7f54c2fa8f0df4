# Round 3: stage sensitivity of the overlapped headline step (timing experiment: SRSGPU_BENCH_SKIP drops a stage's
# launches from the captured step) and a serialised kernel profile of the current code.
set -o pipefail
OUT=gpurun_out/r3v
mkdir -p $OUT
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for s in none encode dmrs,modulate ofdm_mod ofdm_demod chest demod decode encode,dmrs,modulate,ofdm_mod ofdm_demod,chest,demod,decode; do
  SRSGPU_BENCH_SKIP=$([ $s = none ] && echo "" || echo $s) timeout -k 10 200 python bench.py $B > $OUT/skip_$s.json 2> $OUT/skip_$s.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step']*1e3,1), 'us/step')" $OUT/skip_$s.json $s
done
bash tools/gpu/serial_profile.sh r3v/serial
