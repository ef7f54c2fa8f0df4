"""Prints the kernel timeline of consecutive launch groups from a rocprofv3 SQLite trace (rocpd database):
python tools/trace_timeline.py DB [first_group] [nof_groups]. Groups are split at gaps above 100 us."""
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    c = sqlite3.connect(db)
    sym = {r[0]: (r[1] or r[2]) for r in c.execute("select id, kernel_name, display_name from rocpd_info_kernel_symbol")}
    rows = c.execute("select kernel_id, start, end from kernels order by start").fetchall()
    groups, cur = [], []
    for r in rows:
        if cur and r[1] - cur[-1][2] > 100000:
            groups.append(cur)
            cur = []
        cur.append(r)
    groups.append(cur)
    for g in groups[first: first + count]:
        t0 = g[0][1]
        print(f"--- span {(g[-1][2] - t0) / 1000:.1f} us, {len(g)} kernels")
        for k, s, e in g:
            name = re.sub(r"\(.*", "", sym.get(k) or "")
            name = re.sub(r"^_ZN\d+\w*?GLOBAL__N_1\d+", "", name)[:70]
            print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f}  {name}")


if __name__ == "__main__":
    main()
