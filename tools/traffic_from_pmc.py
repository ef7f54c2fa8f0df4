#!/usr/bin/env python3
"""Per-launch HBM traffic of the LDPC decoder kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; they do
not fit one pass on gfx950), written to profiles/ldpc_decode_traffic.json for bench.py's roofline "traffic" field.

FETCH_SIZE is doubled: MI355X_MICROARCH.md (HBM section) - on gfx950 it reports half the bytes of 128-B read
requests. WRITE_SIZE is taken as is. Both are in KB per dispatch (summed over the XCDs by rocprofv3).

    python tools/traffic_from_pmc.py FETCH_DIR WRITE_DIR BENCH_JSON OUT_JSON
"""
import csv
import glob
import json
import sys


def per_dispatch(d, counter, kernel_substr):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    names = {}
    for r in csv.DictReader(open(f)):
        if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel_substr} in {f}")
    avg = sum(vals.values()) / len(vals)
    return avg, len(vals), sorted(set(names.values()))


def main():
    fetch_dir, write_dir, bench_json, out = sys.argv[1:5]
    k = "ldpc_decode_pk_kernel"
    fetch_kb, nf, kn = per_dispatch(fetch_dir, "FETCH_SIZE", k)
    write_kb, nw, _ = per_dispatch(write_dir, "WRITE_SIZE", k)
    bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
    alg = bench["roofline"]["achieved"] * 1e9 * bench["roofline"]["kernel_ms_per_launch"] * 1e-3
    snr = bench["operating_points"][0]["snr_db"]
    res = {
        "kernel": kn[0] if kn else k,
        "workload": bench["roofline"].get("workload_key") or (
            f"{bench['config']['profile']}/S{bench['config']['slots_per_step']}/"
            f"{'noise' if snr is None else f'{snr:g}dB'}"),  # bench.py matches it before using the numbers
        "dispatches_fetch": nf,
        "dispatches_write": nw,
        "fetch_size_kb_raw": fetch_kb,
        "write_size_kb": write_kb,
        "hbm_bytes_per_launch": 2.0 * fetch_kb * 1024.0 + write_kb * 1024.0,
        "algorithmic_bytes_per_launch": alg,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes with --kernel-trace; FETCH_SIZE "
                  "doubled per MI355X_MICROARCH.md (gfx950 reports half the bytes of 128-B read requests), "
                  "WRITE_SIZE as is",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
