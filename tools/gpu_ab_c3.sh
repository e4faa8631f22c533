#!/bin/bash
# A/B of two library builds on the C3 host entry: default vs ab/$1 (SRG_LIB_PATH), three rounds
# usage: tools/gpu_ab_c3.sh LIBNAME TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$2; mkdir -p $O
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then L=$GRAFT_REPO_ROOT/ab/$1; else L=; fi
    SRG_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 5 --no-cpu --no-ri > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || { tail -5 $O/c3_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c3_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['step_ms']['median'], d['breakdown_ms']['ms_scan'], d['device_entry_ms'])"
  done
done
SRG_DEBUG_OVERLAP=1 timeout -k 10 300 python -u bench.py --steps 3 --no-cpu --no-ri --no-verify > $O/c3_dbg.json 2> $O/c3_dbg.err && grep "late loss" $O/c3_dbg.err | tail -4
SRG_DEBUG_OVERLAP=1 timeout -k 10 300 python -u bench.py --steps 3 --no-cpu --no-ri --no-verify > $O/c3dbg.json 2> $O/c3dbg.err && grep "late loss" $O/c3dbg.err | tail -4
