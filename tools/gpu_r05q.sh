#!/bin/bash
# Round 5: catch-up launch sizing A/B (overlap parity first)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05q}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fw_overlap.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --no-verify > $O/c3_new_$i.json 2> $O/c3_new_$i.err || exit 1
  SRG_TMP_CATCHUP_OLD=1 timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --no-verify > $O/c3_old_$i.json 2> $O/c3_old_$i.err || exit 1
done
SRG_DEBUG_OVERLAP=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-ri --no-verify > $O/dbg.json 2> $O/dbg.err || exit 1
grep "last pivot" $O/dbg.err | tail -2
python3 - "$O" <<'PY'
import json,glob,sys
O=sys.argv[1]
for f in sorted(glob.glob(O+"/c3_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); b=d["breakdown_ms"]
    print(f, d["ms_per_step"], "h2d", b["ms_h2d"], "scan", b["ms_scan"])
PY
