#!/bin/bash
# Round 5: 3 vs 4 host-entry scan groups (40/32/7 vs 32/32/8/7), alternating C3 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05g4}; mkdir -p $O
for i in 1 2 3; do
  for g in 3 4; do
    timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --scan-groups $g > $O/c3_g${g}_$i.json 2> $O/c3_g${g}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/c3_g${g}_$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('groups $g', d['ms_per_step'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'd2h', b['ms_d2h'], 'scan+d2h', round(b['ms_scan']+b['ms_d2h'],2), d['verified_rows']['bit_exact'])"
  done
done
