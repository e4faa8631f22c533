#!/bin/bash
# C3 host entry A/B of an environment setting: default vs $1 (e.g. SRG_LOSS_DIRECT=0), three rounds,
# then one SRG_DEBUG_OVERLAP run of each.  usage: tools/gpu_ab_c3env.sh VAR=VALUE TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$2; mkdir -p $O
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then E="$1"; else E=X_UNUSED=0; fi
    env $E timeout -k 10 300 python -u bench.py --steps 5 --no-cpu --no-ri > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || { tail -5 $O/c3_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c3_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['step_ms']['median'], d['breakdown_ms']['ms_scan'], d['device_entry_ms'], d['verified_rows']['bit_exact'])"
  done
done
for v in new base; do
  if [ $v = base ]; then E="$1"; else E=X_UNUSED=0; fi
  env $E SRG_DEBUG_OVERLAP=1 timeout -k 10 300 python -u bench.py --steps 3 --no-cpu --no-ri --no-verify > $O/c3dbg_$v.json 2> $O/c3dbg_$v.err && grep "late loss" $O/c3dbg_$v.err | tail -4
done
