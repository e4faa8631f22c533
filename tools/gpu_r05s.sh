#!/bin/bash
# Round 5: cross-stream hops, value hops (default on one context) vs event waits, C3 host + device entry
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05s}; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --no-verify > $O/c3_val_$i.json 2> $O/c3_val_$i.err || exit 1
  SRG_STREAM_HOPS=events timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --no-verify > $O/c3_evt_$i.json 2> $O/c3_evt_$i.err || exit 1
done
python3 - "$O" <<'PY'
import json,glob,sys
O=sys.argv[1]
for f in sorted(glob.glob(O+"/c3_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); b=d["breakdown_ms"]
    print(f, d["ms_per_step"], "h2d", b["ms_h2d"], "scan", b["ms_scan"], "device", d.get("device_entry_ms"))
PY
