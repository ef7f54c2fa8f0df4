# Bench smoke + SNR sweep of the headline profile (tuning run).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bt
timeout -k 10 300 python bench.py --steps 400 --point-steps 200 --cpu-seconds 4 > gpurun_out/bt/bench.json 2> gpurun_out/bt/bench.err || exit $?
for snr in 16 18 20 22 24 26; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-extra-points --no-cpu-baseline --snr-db $snr > gpurun_out/bt/snr_$snr.json 2>> gpurun_out/bt/bench.err || exit $?
done
