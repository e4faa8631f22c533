#!/bin/bash
# round 4 pass o: catch-up launch size A/B (FW beside the H2D)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04o}
mkdir -p $out
for i in 1 2; do
for w in 768; do
  SRG_CATCHUP_WGS=$w timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri --no-verify > $out/c3_w${w}_$i.json 2> $out/c3_w${w}_$i.err || { echo "c3 $w failed"; tail -10 $out/c3_w${w}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c3_w${w}_$i.json')); b=d['breakdown_ms']; print('w$w', d['ms_per_step'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'total', b['ms_total'])"
done
done
