"""Per-launch PMC averages of the sparse kernel (k_sparse_ds, two-phase; k_sparse_bf, wide labels) from a tools/pmc_sparse.sh output
directory -> profiles/sparse_pmc_latest.json (read by bench.py --graph ba).

usage: python tools/pmc_extract_sparse.py PMC_DIR SOURCE_TEXT [WORKLOAD_KEY]
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB and on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads, so hbm = 2*FETCH + WRITE (an upper
estimate for the sparse kernel, whose label reads are 512-byte wave rows but whose CSR reads are
partly narrow).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d, source = sys.argv[1], sys.argv[2]
    wkey = sys.argv[3] if len(sys.argv) > 3 else None
    # per build: the two-phase kernel runs as two launches (MODE 1: phase 1, MODE 2: phases 2 +
    # output) or one fused launch (MODE 0); a build's counters are the sum over its launches
    tot = collections.defaultdict(float)
    builds = collections.defaultdict(set)
    names = set()
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "k_sparse_ds" not in name and "k_sparse_bf" not in name:
                continue
            names.add(name)
            c = r["Counter_Name"]
            tot[c] += float(r["Counter_Value"])
            m = re.search(r"k_sparse_ds<\s*\w+,\s*\d+,\s*\d+,\s*(\d+)", name)
            if not (m and m.group(1) == "2"):  # one launch per build opens it
                builds[c].add((f, r.get("Dispatch_Id", r.get("Index", ""))))
    avg = {c: tot[c] / max(1, len(builds[c])) for c in tot}
    fetch, write = avg.get("FETCH_SIZE", 0.0), avg.get("WRITE_SIZE", 0.0)
    out = {"source": source, "workload_key": wkey, "kernel": ", ".join(sorted(names)) or None,
           "builds_averaged": len(builds.get("FETCH_SIZE", ())),
           "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "hbm_bytes_per_launch": int((2 * fetch + write) * 1024),
           "hbm_bytes_per_launch_low": int((fetch + write) * 1024),
           "note": "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB->B, gfx950 half-count correction); "
                   "_low = FETCH_SIZE + WRITE_SIZE without the correction"}
    for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
              "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
        if c in avg:
            out[c] = avg[c]
    p = os.path.join(ROOT, "profiles", "sparse_pmc_latest.json")
    json.dump(out, open(p, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
