# Kernel durations with the legs serialised and no cross-step pipelining (no kernel overlaps another), for per-kernel
# comparisons; output under gpurun_out/$1.
set -euo pipefail
OUT=gpurun_out/${1:-serial}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/stats" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-extra-points --steps 40 --warmup 4 --serial-legs --no-pipeline \
  ${2:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
find "$OUT" -name "*kernel_trace.csv" -delete
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f"{r['Name'][:60]:60s} {float(r['AverageNs'])/1000:8.1f} us x {r['Calls']}")
PY
