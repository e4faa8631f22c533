#!/bin/bash
# round 4 pass k: FW beside the H2D with sub-tile chain lines (line split 1 / 2 / 4), and without overlap
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04k}
mkdir -p $out
for i in 1 2; do
for cfg in "s1:--fw-overlap 1 --fw-line-split 1" "s2:--fw-overlap 1 --fw-line-split 2" "s4:--fw-overlap 1 --fw-line-split 4" "o0s2:--fw-overlap 0 --fw-line-split 2"; do
  name=${cfg%%:*}; args=${cfg#*:}
  SRG_DEBUG_OVERLAP=1 timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-verify --no-ri $args > $out/c3_${name}_$i.json 2> $out/c3_${name}_$i.err || { echo "c3 $name failed"; tail -20 $out/c3_${name}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c3_${name}_$i.json')); b=d['breakdown_ms']; print('$name', d['ms_per_step'], 'h2d', b['ms_h2d'], 'fw', b['ms_fw'], 'scan', b['ms_scan'], 'total', b['ms_total'], 'dev', d['device_entry_ms'])"
  grep "last pivot" $out/c3_${name}_$i.err | tail -1
done
done
