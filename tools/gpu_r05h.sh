#!/bin/bash
# Round 5: tight_v6 parity vs tight_v5, then C3 A/B (scan kernel 5 vs 6) with rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05h}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_scan_v6.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for k in 6 5; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --scan-kernel $k > $O/c3_k$k.json 2> $O/c3_k$k.err || { tail $O/c3_k$k.err; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof6 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ri --no-verify --scan-kernel 6 > $O/prof6.log 2>&1 || { tail $O/prof6.log; exit 1; }
python3 - "$O" <<'PY'
import json,glob,sys
O=sys.argv[1]
for f in sorted(glob.glob(O+"/c3_k*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); b=d["breakdown_ms"]; print(f, d["ms_per_step"], b["ms_h2d"], b["ms_scan"], b["ms_d2h"], d.get("verified_rows"))
for f in glob.glob(O+"/prof6/**/*kernel_stats.csv", recursive=True):
    for l in open(f).read().splitlines()[:12]: print(l[:160])
PY
