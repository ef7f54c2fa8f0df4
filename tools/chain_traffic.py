#!/usr/bin/env python3
"""HBM traffic per launch of the signal-chain kernels (and the decoder) from two rocprofv3 PMC passes of the bench
(FETCH_SIZE, WRITE_SIZE: separate passes on gfx950), against the bench's algorithmic bytes per launch
(bench.py "stage_algorithmic_bytes": each byte a stage must read or write, once).

FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM section: gfx950 reports half the bytes of wide coalesced reads; the
narrower accesses of these kernels are uncalibrated, so the doubled value is an upper estimate of the read bytes and
the raw value a lower one - both are kept). WRITE_SIZE is taken as is. Both come in KB per dispatch.

    python tools/chain_traffic.py FETCH_DIR WRITE_DIR BENCH_JSON [KERNEL_STATS_CSV] > traffic.json
"""
import csv
import glob
import json
import sys

# bench stage -> kernel-name prefixes whose dispatches make up the stage's launch (one launch per step each)
STAGES = {
    "ofdm_modulate": ["ofdm_modulate_kernel"],
    "ofdm_demodulate": ["ofdm_demodulate_kernel"],
    "pusch_channel_estimate": ["pusch_chest_kernel"],
    "pusch_demodulate": ["pusch_demodulate_kernel"],
    "pdsch_encode": ["pdsch_encode_packed_kernel", "pdsch_encode_kernel", "tb_crc_kernel"],
    "pdsch_dmrs_modulate": ["pdsch_dmrs_kernel", "pdsch_modulate_kernel"],
}


def short(name):
    for ns in ("srsgpu::(anonymous namespace)::", "void "):
        name = name.replace(ns, "")
    return name.split("(")[0]


def per_kernel(d, counter):
    """Per kernel: (average counter value per dispatch, dispatches, average dispatch duration in us). Counter
    collection runs the dispatches one at a time, so the durations are the kernels' isolated ones."""
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    disp, dur = {}, {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        key = (short(r["Kernel_Name"]), r["Dispatch_Id"])
        disp[key] = disp.get(key, 0.0) + float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    out = {}
    for key, v in disp.items():
        s, n, t = out.get(key[0], (0.0, 0, 0.0))
        out[key[0]] = (s + v, n + 1, t + dur[key])
    return {k: (s / n, n, t / n) for k, (s, n, t) in out.items()}


def durations(stats_csv):
    """Average duration (us) per kernel from a rocprofv3 --stats kernel_stats.csv (concurrent kernels overlap there)."""
    res = {}
    if stats_csv:
        for r in csv.DictReader(open(stats_csv)):
            res[short(r["Name"])] = float(r["AverageNs"]) / 1e3
    return res


def main():
    fetch_dir, write_dir, bench_json = sys.argv[1:4]
    stats = durations(sys.argv[4] if len(sys.argv) > 4 else None)
    fetch = per_kernel(fetch_dir, "FETCH_SIZE")  # its dispatch durations are the isolated kernel times
    write = per_kernel(write_dir, "WRITE_SIZE")
    bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
    alg_stage = bench.get("stage_algorithmic_bytes", {})
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes with --kernel-trace of the "
                     "bench's short profiled run; per dispatch, averaged per kernel; fetch doubled (gfx950, "
                     "MI355X_MICROARCH.md) as the upper estimate",
           "stages": {}}
    for stage, prefixes in STAGES.items():
        ks = sorted(k for k in set(fetch) | set(write) if any(k.startswith(p) for p in prefixes))
        if not ks:
            continue
        # The stage's per-step kernels only: a kernel dispatched far fewer times belongs to the bench's other
        # workloads or operating points (e.g. the byte encoder of the test-mode workload), not to the headline launch.
        most = max(fetch.get(k, (0.0, 0, 0.0))[1] for k in ks)
        ks = [k for k in ks if fetch.get(k, (0.0, 0, 0.0))[1] * 2 >= most]
        f_kb = sum(fetch.get(k, (0.0, 0))[0] for k in ks)
        w_kb = sum(write.get(k, (0.0, 0))[0] for k in ks)
        alg = alg_stage.get(stage)
        hbm_hi = (2.0 * f_kb + w_kb) * 1024.0
        hbm_lo = (f_kb + w_kb) * 1024.0
        e = {"kernels": {k: {"fetch_kb_raw": fetch.get(k, (0.0, 0, 0.0))[0], "write_kb": write.get(k, (0.0, 0, 0.0))[0],
                             "dispatches": fetch.get(k, (0.0, 0, 0.0))[1],
                             "isolated_us": fetch.get(k, (0.0, 0, 0.0))[2], "overlapped_avg_us": stats.get(k)}
                         for k in ks},
             "hbm_bytes_per_launch": hbm_hi, "hbm_bytes_per_launch_fetch_undoubled": hbm_lo,
             "write_bytes_per_launch": w_kb * 1024.0, "read_bytes_per_launch": 2.0 * f_kb * 1024.0,
             "algorithmic_bytes_per_launch": alg}
        if alg:
            e["traffic_ratio"] = hbm_hi / alg
            e["traffic_ratio_fetch_undoubled"] = hbm_lo / alg
        us = sum(fetch.get(k, (0.0, 0, 0.0))[2] for k in ks)
        if us > 0 and alg:
            e["isolated_us"] = us
            e["algorithmic_gbps_isolated"] = alg / (us * 1e-6) / 1e9
            e["hbm_fraction_of_8tbs_isolated"] = alg / (us * 1e-6) / 8e12
        res["stages"][stage] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
