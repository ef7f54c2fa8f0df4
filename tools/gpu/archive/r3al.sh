# Round 3: step shape with the leg graphs: slots per step x input sets (headline bench).
set -o pipefail
OUT=gpurun_out/r3al
mkdir -p $OUT
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
run() {
  timeout -k 10 240 python bench.py $B $2 > $OUT/$1.json 2> $OUT/$1.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), round(d['ms_per_step'],4), d['ldpc_avg_iterations'])" $OUT/$1.json
}
for i in 1 2; do
  run s32k9_$i ""
  run s40k9_$i "--slots-per-step 40"
  run s48k9_$i "--slots-per-step 48"
  run s24k12_$i "--slots-per-step 24 --input-sets 12"
  run s48k7_$i "--slots-per-step 48 --input-sets 7"
done
