#!/usr/bin/env python3
"""Kernel overlap of a bench run from a rocprofv3 --kernel-trace CSV: busy time vs the sum of kernel durations,
time at each concurrency level, and the kernel intervals of a window of the timed loop (the graph replays).
Usage: overlap_from_trace.py <kernel_trace.csv> <out.json> [window_us]"""
import csv
import json
import re
import sys


def short(name):
    m = re.search(r"::(\w+(<[^>]*>)?)\(", name)
    return m.group(1) if m else name.split("(")[0][-60:]


def main():
    path, out = sys.argv[1], sys.argv[2]
    window_us = float(sys.argv[3]) if len(sys.argv) > 3 else 600.0
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    # The timed loop: the longest run of srsgpu kernels without a gap above 1 ms, taken from its middle.
    srs = [x for x in iv if "srsgpu" in x[2] or x[2].startswith(("ldpc", "pdsch", "pusch", "ofdm", "rate", "tb_"))]
    runs, cur = [], [srs[0]]
    for a, b in zip(srs, srs[1:]):
        if b[0] - max(e for _, e, _ in cur[-50:]) > 1_000_000:
            runs.append(cur)
            cur = []
        cur.append(b)
    runs.append(cur)
    run = max(runs, key=len)
    t0, t1 = run[0][0], max(e for _, e, _ in run)
    events = sorted([(s, 1) for s, _, _ in run] + [(e, -1) for _, e, _ in run])
    level, last, hist = 0, t0, {}
    for t, d in events:
        hist[level] = hist.get(level, 0) + (t - last)
        level += d
        last = t
    busy = sum(v for k, v in hist.items() if k > 0)
    total_kernel = sum(e - s for s, e, _ in run)
    mid = t0 + (t1 - t0) // 2
    win = [x for x in run if x[1] > mid and x[0] < mid + window_us * 1000]
    res = {
        "source": "rocprofv3 --kernel-trace of bench.py (timed loop: graph replays of the pipelined input sets)",
        "span_us": (t1 - t0) / 1e3,
        "kernels": len(run),
        "busy_us": busy / 1e3,
        "sum_kernel_us": total_kernel / 1e3,
        "overlap_factor": total_kernel / max(busy, 1),
        "time_fraction_by_concurrency": {str(k): v / max(t1 - t0, 1) for k, v in sorted(hist.items())},
        "window_us": window_us,
        "window": [{"kernel": n, "start_us": round((s - mid) / 1e3, 2), "end_us": round((e - mid) / 1e3, 2)}
                   for s, e, n in win],
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "window"}, indent=1))


if __name__ == "__main__":
    main()
