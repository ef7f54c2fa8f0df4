# Round 3: where the one-codeblock decoder's issue goes (2048 Z = 288 codeblocks, 6 iterations, no CRC): VALU / LDS
# activity, LDS latency and FIFOs, instruction fetch, instruction cache. One PMC pass per counter group.
set -o pipefail
mkdir -p gpurun_out/r3m
export TMPDIR=/tmp
R=$(pwd)
run() {
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $2 -d "$R/gpurun_out/r3m/$1" -o run --output-format csv -- python3 "$R/tools/decoder_scaling.py" --z 288 --cols 30 --iters 6 --no-crc --sizes 2048 > gpurun_out/r3m/$1.log 2>&1
}
run a "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS GRBM_GUI_ACTIVE" || exit $?
run b "SQ_IFETCH SQ_IFETCH_LEVEL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE" || exit $?
run c "SQC_ICACHE_BUSY_CYCLES SQC_TC_INST_REQ SQC_TC_STALL GRBM_GUI_ACTIVE" || exit $?
python3 - <<'PY'
import csv, glob, collections
for p in "abc":
    fs = glob.glob(f"gpurun_out/r3m/{p}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print(p, "no csv"); continue
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(fs[0])):
        if "ldpc_decode" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    L = max(n.values()) if n else 1
    print(p, " ".join(f"{k}={acc[k]/L:.4g}" for k in sorted(acc)))
PY
find gpurun_out/r3m -name "*.csv" -size +2M -delete
