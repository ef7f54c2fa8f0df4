#!/usr/bin/env python3
"""Merges one workload's decoder traffic summary (tools/traffic_from_pmc.py) and SQ summary (tools/sq_summary.py) into
profiles/ldpc_decode_traffic.json and profiles/sq_valu.json, keyed by the bench workload (bench.py reads them).

    python tools/merge_profiles.py TRAFFIC_JSON SQ_JSON SOURCE_NOTE
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def merge(path, entry, note):
    with open(path) as f:
        j = json.load(f)
    key = entry["workload"]
    entry = dict(entry, source=note)
    j.setdefault("by_workload", {})[key] = entry
    with open(path, "w") as f:
        json.dump(j, f, indent=1)
    print(f"{os.path.basename(path)}: {key} <- {note}")


if __name__ == "__main__":
    traffic, sq, note = sys.argv[1:4]
    merge(os.path.join(ROOT, "profiles", "ldpc_decode_traffic.json"), json.load(open(traffic)), note)
    merge(os.path.join(ROOT, "profiles", "sq_valu.json"), json.load(open(sq)), note)
