#!/usr/bin/env bash
# Round 4: hardware-queue sweep of the headline step (4 = HIP default, 6, 8), no CPU baseline.
set -o pipefail
mkdir -p gpurun_out
PB="--no-cpu-baseline --no-extra-points --no-extra-workloads --steps 2000 --warmup 20"
for q in 4 6 8 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py $PB > gpurun_out/r4t_q$q.json 2> gpurun_out/r4t_q$q.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']))" gpurun_out/r4t_q$q.json $q >> gpurun_out/r4t_summary.txt
done
