"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd sqlite) into profiles/.

usage: python tools/rocpd_stats.py DB OUT_PREFIX [KERNEL_SUBSTR]
writes OUT_PREFIX_kernel_stats.csv (per kernel: calls, total/avg/min/max us, %) and
OUT_PREFIX_dominant.json: the KERNEL_SUBSTR kernel's dispatches grouped by grid size, so the
bulk (largest-grid) launches can be compared with bench.py's HIP-event average.
"""
import collections
import csv
import json
import sqlite3
import sys


def main():
    db, prefix = sys.argv[1], sys.argv[2]
    sub = sys.argv[3] if len(sys.argv) > 3 else None
    c = sqlite3.connect(db)
    cur = c.execute("select * from kernels limit 1")
    cols = [d[0] for d in cur.description]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    q = f"select {name_col}, start, end, grid_x, grid_y, grid_z from kernels"
    per = collections.defaultdict(list)
    grids = collections.defaultdict(list)
    for name, s, e, gx, gy, gz in c.execute(q):
        d = (e - s) / 1e3  # ns -> us
        per[name].append(d)
        if sub and sub in name:
            grids[(name, gx * gy * gz)].append(d)
    tot = sum(sum(v) for v in per.values())
    rows = sorted(per.items(), key=lambda kv: -sum(kv[1]))
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalUs", "AverageUs", "MinUs", "MaxUs", "Percentage"])
        for name, v in rows:
            w.writerow([name, len(v), round(sum(v), 3), round(sum(v) / len(v), 3), round(min(v), 3),
                        round(max(v), 3), round(100 * sum(v) / tot, 3)])
    if sub:
        out = {"kernel_substr": sub, "by_grid": []}
        for (name, g), v in sorted(grids.items(), key=lambda kv: -kv[0][1]):
            out["by_grid"].append({"kernel": name[:100], "grid_threads": g, "calls": len(v),
                                   "avg_us": round(sum(v) / len(v), 3)})
        json.dump(out, open(prefix + "_dominant.json", "w"), indent=1)
        print(json.dumps(out["by_grid"][:4], indent=1))
    for name, v in rows[:8]:
        print(f"{sum(v) / 1e3:9.2f} ms {len(v):5d} calls  {name[:90]}")


if __name__ == "__main__":
    main()
