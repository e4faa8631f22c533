"""rocprofv3 kernel-trace average of the FW bulk launches bench.py times (round 4).

With the FW beside the H2D, the early bulk launches cover only the block-rows that have landed
(same grid, fewer live tiles) and the bench's HIP events time only the launches after every row
is in (maxI = nb - 1, k1 < nb).  Those are the launches that start after the build's last
fw_catchup (the last late rows caught up), minus the build's final pivot.
usage: python tools/rocprof_full_launches.py KERNEL_TRACE_CSV"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    bulk = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "fw_bulk_lb" in r["Kernel_Name"])
    cu = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "fw_catchup" in r["Kernel_Name"])
    builds = [[bulk[0]]]
    for a, b in zip(bulk, bulk[1:]):
        if b[0] - a[0] > 2e6:  # builds are > 2 ms apart
            builds.append([])
        builds[-1].append(b)
    full, per = [], []
    for b in builds:
        t0, t1 = b[0][0], b[-1][1]
        last_cu = max([c[1] for c in cu if t0 - 5e6 <= c[0] <= t1] or [t0])
        f = [(e - s) / 1e3 for s, e in b[:-1] if s >= last_cu]
        full += f
        per.append(len(f))
    allb = [(e - s) / 1e3 for s, e in bulk]
    print(f"builds {len(builds)}, bulk launches {len(bulk)} (all: {sum(allb) / len(allb):.1f} us avg)")
    print(f"full launches per build {per}")
    print(f"rocprof average of the full launches: {sum(full) / len(full):.1f} us over {len(full)}")


if __name__ == "__main__":
    main()
