"""Per-launch PMC averages for one kernel from a PMC output directory (tools/pmc_*.sh).
usage: python tools/pmc_kernel.py PMC_DIR KERNEL_SUBSTR"""
import collections
import csv
import glob
import os
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for c, v in sorted(acc.items()):
        print(f"{c:24s} launches={len(v):4d} avg={sum(v) / len(v):.4g}")


if __name__ == "__main__":
    main()
