#!/bin/bash
# round 4 pass i: fresh-table page-locking (prefault A/B), RoutingInfo build breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04i}
mkdir -p $out
for pf in 1 0; do
  SRG_PREFAULT=$pf timeout -k 10 200 python3 -u tools/cold_probe2.py > $out/cold_pf$pf.json 2> $out/cold_pf$pf.err && echo "pf$pf $(cat $out/cold_pf$pf.json)" || { echo "cold $pf failed"; tail -5 $out/cold_pf$pf.err; exit 1; }
  SRG_PREFAULT=$pf SRG_DEBUG_CODEC=1 timeout -k 10 200 python3 -u tools/ri_probe.py > $out/ri_pf$pf.json 2> $out/ri_pf$pf.err && echo "ri pf$pf $(cat $out/ri_pf$pf.json)" || { echo "ri $pf failed"; tail -5 $out/ri_pf$pf.err; exit 1; }
  grep codec $out/ri_pf$pf.err | head -4
done
