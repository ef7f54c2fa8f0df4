"""Per-kernel VALU issue rate and wave-state breakdown from a rocprofv3 --pmc pass with SQ_INSTS_VALU, SQ_WAVES,
SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_INSTS_LDS (run_counter_collection.csv).
VALU peak: 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md) = 1.23 T instr/s."""
import collections
import csv
import sys

PEAK = 1024 * 2.4e9 / 2


def main(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("srsgpu::(anonymous namespace)::", "").replace("void ", "")
        if "rocclr" in n or "at::" in n or "rocsolver" in n or "rocblas" in n or "Cijk" in n:
            continue
        k = n.split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for k, c in sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]].values())):
        d = {cn: sum(v) / len(v) for cn, v in c.items()}
        t = sum(dur[k].values()) / len(dur[k]) * 1e-9
        wc = d["SQ_WAVE_CYCLES"]
        row = {"us": t * 1e6, "valu_instr": d["SQ_INSTS_VALU"], "waves": d["SQ_WAVES"],
               "valu_issue_frac": d["SQ_INSTS_VALU"] / t / PEAK, "wait_any": d["SQ_WAIT_ANY"] / wc,
               "wait_inst_any": d["SQ_WAIT_INST_ANY"] / wc, "active_inst_any": d["SQ_ACTIVE_INST_ANY"] / wc,
               "lds_instr": d.get("SQ_INSTS_LDS", 0.0)}
        out[k] = row
        print(f"{k:36s} {row['us']:7.1f} us  VALU {row['valu_instr'] / 1e6:7.2f} M  issue {row['valu_issue_frac']:5.1%}"
              f"  waves {row['waves']:7.0f}  wait {row['wait_any']:4.0%}  stall {row['wait_inst_any']:4.0%}"
              f"  active {row['active_inst_any']:4.0%}")
    return out


if __name__ == "__main__":
    import json
    res = main(sys.argv[1])
    if len(sys.argv) > 3:  # sq_summary.py CSV OUT_JSON BENCH_JSON: keyed by the bench workload (bench.py checks it)
        bench = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
        snr = bench["operating_points"][0]["snr_db"]
        res = {"workload": bench["roofline"].get("workload_key") or (
            f"{bench['config']['profile']}/S{bench['config']['slots_per_step']}/"
            f"{'noise' if snr is None else f'{snr:g}dB'}"), "kernels": res}
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)
