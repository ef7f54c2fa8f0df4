# Round 3: --leg-graphs (DL and UL legs as two graphs on two streams per input set) over the number of input sets.
set -o pipefail
OUT=gpurun_out/r3ai3
mkdir -p $OUT
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
run() {  # name, args
  timeout -k 10 200 python bench.py $B $2 > $OUT/$1.json 2> $OUT/$1.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), d['ldpc_avg_iterations'])" $OUT/$1.json
}
for i in 1 2; do
  run base7_$i "--input-sets 7"
  for k in 7 8 9 10 11 14; do
    run leg${k}_$i "--leg-graphs --input-sets $k"
  done
done
