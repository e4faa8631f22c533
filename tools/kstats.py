"""Print the rocprofv3 kernel-stats rows of the named kernels: calls, average and total time."""
import csv
import sys

pats = sys.argv[2:] or ["tight_v5", "k_loss_rows", "k_v5_fill", "k_ess_mask", "k_extract", "fw_bulk_lb"]
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(p in n for p in pats):
        print(f"{n.split('(')[0][-40:]:40s} calls {int(r['Calls']):6d} avg_us {float(r['AverageNs'])/1e3:9.1f} total_ms {float(r['TotalDurationNs'])/1e6:9.2f}")
