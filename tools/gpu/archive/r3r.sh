# Round 3: full GPU parity suite (one pytest process), then smoke() and the driver-shaped bench command.
set -o pipefail
mkdir -p gpurun_out/r3r
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3r/gpu_tests.log 2>&1
rc=$?
tail -6 gpurun_out/r3r/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3r/smoke.log 2>&1 || exit $?
tail -3 gpurun_out/r3r/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r3r/bench_driver.json 2> gpurun_out/r3r/bench_driver.err || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', round(d['value']), d['steps'], round(d['config']['timed_region_s'],2))" gpurun_out/r3r/bench_driver.json
