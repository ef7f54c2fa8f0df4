# Round 3: SQ counters of the one-codeblock (PK4=0) and multi-codeblock (PK4=1) decoder on 2048 Z = 288 codeblocks
# (8-layer span, 6 iterations, no CRC): VALU / LDS instructions, LDS bank conflicts, wait and issue cycles.
set -o pipefail
mkdir -p gpurun_out/r3j
export TMPDIR=/tmp
R=$(pwd)
for v in 0 1; do
  SRSGPU_DECODER_PK4=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d "$R/gpurun_out/r3j/pmc_$v" -o run --output-format csv -- python3 "$R/tools/decoder_scaling.py" --z 288 --cols 30 --iters 6 --no-crc --sizes 2048 > gpurun_out/r3j/run_$v.log 2>&1 || exit $?
  cat gpurun_out/r3j/run_$v.log | grep -v amdgpu.ids
done
python3 - <<'PY'
import csv, glob, collections
for v in (0, 1):
    f = glob.glob(f"gpurun_out/r3j/pmc_{v}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "ldpc_decode" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            n["launches"] += 1
    L = max(n["launches"], 1)
    print(f"PK4={v} launches={L} " + " ".join(f"{k}={acc[k]/L:.4g}" for k in sorted(acc)))
PY
find gpurun_out/r3j -name "*.csv" -size +2M -delete
