#!/usr/bin/env python3
"""Kernels per bench step from a rocprofv3 kernel trace (tools/gpu/ktrace.sh).

The timed loop replays one UL decoder launch per step, so the decoder's dispatches mark the steps. The script takes
the longest run of decoder dispatches whose start-to-start gaps stay below 4x their median (the timed loop, not the
eager passes), and reports for every kernel name: dispatches per step, mean duration and busy time per step.
Usage: trace_per_step.py kernel_trace.csv[.gz] [decoder-name-substring]
"""
import csv
import gzip
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "ldpc_decode_pk_kernel"
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rt") as f:
        rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(f)]
    rows.sort()
    dec = [r for r in rows if key in r[2]]
    gaps = [b[0] - a[0] for a, b in zip(dec, dec[1:])]
    med = statistics.median(gaps)
    best, cur = (0, 0), 0
    for i, g in enumerate(gaps):
        cur = cur + 1 if g < 4 * med else 0
        if cur > best[1] - best[0]:
            best = (i - cur + 1, i + 1)
    i0, i1 = best
    t0, t1 = dec[i0][0], dec[i1][0]
    steps = i1 - i0
    per = defaultdict(lambda: [0, 0])
    for s, e, n in rows:
        if t0 <= s < t1:
            per[n][0] += 1
            per[n][1] += e - s
    print(f"timed window: {steps} steps, {(t1 - t0) / steps / 1e3:.1f} us per step (start to start)")
    print(f"{'per step':>9} {'mean us':>9} {'busy us/step':>13}  kernel")
    for n, (c, d) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{c / steps:9.2f} {d / c / 1e3:9.1f} {d / steps / 1e3:13.1f}  {n[:110]}")


if __name__ == "__main__":
    main()
