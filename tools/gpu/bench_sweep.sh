# Bench sweep over step shapes: bench_sweep.sh "<args 1>" "<args 2>" ... (one line per configuration).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
i=0
for a in "$@"; do
  i=$((i + 1))
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra-points $a > gpurun_out/sweep/$i.json 2>> gpurun_out/sweep/err.log || exit $?
  python -c "import json; b=json.loads(open('gpurun_out/sweep/$i.json').read().strip().splitlines()[-1]); print('$a |', round(b['value']), round(b['ms_per_step'],4), round(b['roofline']['kernel_ms_per_launch'],4), b['pusch_tb_success_rate'], round(b['ldpc_avg_iterations'],2), round(b['config']['working_set_mb']))"
done
