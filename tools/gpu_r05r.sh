#!/bin/bash
# Round 5: simulated ranks 8:0 / 8:7, XCD tile order on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05r}; mkdir -p $O
for i in 1 2; do for sr in 8:7 8:0; do for x in 1 0; do
  timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr --fw-xcd-order $x > $O/sim_${sr/:/_}_x${x}_$i.json 2> $O/sim_${sr/:/_}_x${x}_$i.err || { tail -5 $O/sim_${sr/:/_}_x${x}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sim_${sr/:/_}_x${x}_$i.json')); b=d['breakdown_ms']; print('$sr x$x', d['ms_per_step'], 'fw', b['ms_fw'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'])"
done; done; done
