#!/bin/bash
# Round 5: chain line split at sim 8:0 with the quadrant bulk: 4 (default, 32 x 32) vs 2 (quadrants)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05s2}; mkdir -p $O
for i in 1 2; do
  for sp in 4 2; do
    timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --simulate-rank 8:0 --fw-line-split $sp > $O/sim8_split${sp}_$i.json 2> $O/sim8_split${sp}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/sim8_split${sp}_$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('split $sp', d['ms_per_step'], 'fw', b['ms_fw'])"
  done
done
