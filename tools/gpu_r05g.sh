#!/bin/bash
# Round 5: the key-D2H / table-pool tests and the parity file, then the default bench line (C3) and
# a C3 A/B of the key D2H
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05g}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_routing_info_keys.py tests/test_gpu_parity.py tests/test_fw_overlap.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri > $O/c3_keys_$i.json 2> $O/c3_keys_$i.err || exit 1
  SRG_NO_KEY_D2H=1 timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri > $O/c3_u64_$i.json 2> $O/c3_u64_$i.err || exit 1
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/%s/c3_*.json" % "${1:-r05g}")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["ms_per_step"], d.get("breakdown_ms",{}).get("ms_h2d"), d.get("breakdown_ms",{}).get("ms_d2h"))
PY
