# Instruction-cache counters of the bench's kernels (one PMC pass, kernel trace); summary per kernel.
set -euo pipefail
OUT=gpurun_out/${1:-icache}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES -d "$R/$OUT/pmc" \
  -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-extra-points --steps 20 --warmup 4 --min-time 0 --no-extra-workloads \
  ${2:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:50]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES":
        n[k] += 1
for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQC_ICACHE_MISSES", 0))[:12]:
    c = max(n[k], 1)
    print(f"{k:50s} launches {c:4d} misses/launch {v['SQC_ICACHE_MISSES']/c:10.0f} hits/launch {v['SQC_ICACHE_HITS']/c:10.0f} ifetch/launch {v['SQ_IFETCH']/c:10.0f} waves {v['SQ_WAVES']/c:8.0f}")
PY
find "$OUT" -name "*.csv" -size +2M -delete
