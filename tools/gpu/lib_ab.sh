# A/B of library builds (SRSGPU_LIB) on one bench configuration: lib_ab.sh "<bench args>" dir1 dir2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/libab
args=$1; shift
for d in "$@"; do
  SRSGPU_LIB=$PWD/srsran-5g_amd/$d/libsrsgpu_phy.so timeout -k 10 200 python bench.py --steps 1000 --no-cpu-baseline --no-extra-points $args > gpurun_out/libab/$d.json 2>> gpurun_out/libab/err.log || exit $?
  python -c "import json; b=json.loads(open('gpurun_out/libab/$d.json').read().strip().splitlines()[-1]); print('$d', round(b['value']), round(b['ms_per_step'],4), round(b['roofline']['kernel_ms_per_launch'],4), b['pusch_tb_success_rate'], b['ldpc_avg_iterations'], {k: round(v * 1e3, 1) for k, v in b['stage_ms_per_step'].items()})"
done
