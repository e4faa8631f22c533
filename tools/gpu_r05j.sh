#!/bin/bash
# Round 5: FW bulk XCD Z-order tile dealing -- parity, C3 A/B, FETCH/WRITE PMC of fw_bulk_lb
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05j}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fw_xcd_order.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do for x in 1 0; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --fw-xcd-order $x > $O/c3_x${x}_$i.json 2> $O/c3_x${x}_$i.err || { tail $O/c3_x${x}_$i.err; exit 1; }
done; done
for x in 1 0; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    SRG_STREAM_HOPS=events timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_x$x/$ctr -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-profile --no-ri --no-verify --fw-overlap 0 --fw-xcd-order $x > $O/pmc_x${x}_$ctr.log 2>&1 || { tail $O/pmc_x${x}_$ctr.log; exit 1; }
  done
done
python3 - "$O" <<'PY'
import json,glob,sys,subprocess
O=sys.argv[1]
for f in sorted(glob.glob(O+"/c3_x*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); b=d["breakdown_ms"]; r=d["roofline"]
    print(f, d["ms_per_step"], b["ms_h2d"], b["ms_scan"], "bulk_avg_ms", r["avg_launch_ms"], "frac", r["frac"])
for x in (1, 0):
    print("xcd_order", x); subprocess.run(["python3", "tools/pmc_kernel.py", f"{O}/pmc_x{x}", "fw_bulk_lb"])
PY
