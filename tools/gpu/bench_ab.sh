# A/B of bench options: each argument string is one bench run (short, no CPU baseline, no extra points).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
i=0
for a in "$@"; do
  timeout -k 10 200 python bench.py --steps 2000 --no-cpu-baseline --no-extra-points $a > gpurun_out/ab/run$i.json 2>> gpurun_out/ab/err.log || exit $?
  python -c "import json,sys; b=json.loads(open('gpurun_out/ab/run$i.json').read().strip().splitlines()[-1]); print('$a', round(b['value']), round(b['ms_per_step'],4), round(b['roofline']['kernel_ms_per_launch'],4), b['pusch_tb_success_rate'])"
  i=$((i+1))
done
