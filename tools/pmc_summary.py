"""Aggregate a rocprofv3 --pmc counter_collection.csv into per-kernel averages per dispatch (small enough to copy
back from the GPU box). Usage: python tools/pmc_summary.py <counter_collection.csv> [kernel-substring ...]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(float))
    dispatches = defaultdict(set)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if keys and not any(k in name for k in keys):
                continue
            short = re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0][-90:]
            acc[short][row["Counter_Name"]] += float(row["Counter_Value"])
            dispatches[short].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    for k in sorted(acc):
        n = max(1, len(dispatches[k]))
        vals = " ".join(f"{c}={v / n:.4g}" for c, v in sorted(acc[k].items()))
        print(f"{k} dispatches={n} {vals}")


if __name__ == "__main__":
    main()
