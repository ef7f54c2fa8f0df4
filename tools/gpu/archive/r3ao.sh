# Round 3: hardware queues per process with the leg-graph structure (headline bench).
set -o pipefail
OUT=gpurun_out/r3ao
mkdir -p $OUT
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for i in 1 2; do
  for q in 4 3 6 5; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py $B > $OUT/q${q}_$i.json 2> $OUT/q${q}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']))" $OUT/q${q}_$i.json
  done
done
