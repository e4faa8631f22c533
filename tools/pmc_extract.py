"""Per-launch PMC averages of the dominant FW kernel (the bulk phase-3 launches) from a
tools/pmc_fw.sh output directory -> profiles/fw_pmc_latest.json (read by bench.py).

usage: python tools/pmc_extract.py PMC_DIR SOURCE_TEXT [WORKLOAD_KEY] [KERNEL_SUBSTR]
WORKLOAD_KEY is bench.py's key of the run the passes profiled (bench.py reports the traffic only
for a run with the same key); KERNEL_SUBSTR defaults to fw_bulk_lb (the symmetric bulk tile).
HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB and on
gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so hbm = 2*FETCH + WRITE.
The bulk launches are the largest-grid dispatches of that kernel (grid >= 90% of the maximum).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d, source = sys.argv[1], sys.argv[2]
    wkey = sys.argv[3] if len(sys.argv) > 3 else None
    ksub = sys.argv[4] if len(sys.argv) > 4 else "fw_bulk_lb<"
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    grids = collections.defaultdict(int)
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if ksub not in name or "pair" in name:
                continue
            g = int(r["Grid_Size"])
            grids[name] = max(grids[name], g)
            per[(name, g)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    name = max(grids, key=lambda k: grids[k])
    gmax = grids[name]
    acc = collections.defaultdict(list)
    launches = 0
    for (n, g), cs in per.items():
        if n != name or g < 0.9 * gmax:
            continue
        for c, v in cs.items():
            acc[c] += v
        launches = max(launches, len(cs.get("FETCH_SIZE", [])))
    avg = {c: sum(v) / len(v) for c, v in acc.items()}
    out = {"source": source, "workload_key": wkey, "kernel": name[:90], "grid_max": gmax, "launches_averaged": launches,
           "FETCH_SIZE_KiB": avg.get("FETCH_SIZE"), "WRITE_SIZE_KiB": avg.get("WRITE_SIZE"),
           "hbm_bytes_per_launch": int((2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0)) * 1024),
           "note": "hbm_bytes = 2*FETCH_SIZE (gfx950 reports half of wide coalesced reads, MI355X_MICROARCH.md) "
                   "+ WRITE_SIZE, KiB->B; algorithmic per launch = the C tiles read + written (+ panels, L2-resident)"}
    for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
              "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES"):
        if c in avg:
            out[c] = avg[c]
    p = os.path.join(ROOT, "profiles", "fw_pmc_latest.json")
    json.dump(out, open(p, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
