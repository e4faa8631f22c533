#!/bin/bash
# A/B of two library builds on C4: default vs ab/$1 (SRG_LIB_PATH), two rounds; extra env in ABENV
# usage: tools/gpu_ab_lib.sh LIBNAME TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$2; mkdir -p $O
for i in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then L=$GRAFT_REPO_ROOT/ab/$1; else L=; fi
    env $ABENV SRG_LIB_PATH=$L SRG_DEBUG_SPARSE=1 timeout -k 10 300 python -u bench.py --config c4 --entry device --steps 3 --no-cpu --no-ri > $O/c4_${v}_$i.json 2> $O/c4_${v}_$i.err || { tail -5 $O/c4_${v}_$i.err; exit 1; }
    echo "$v $(python3 -c "import json; print(json.loads(open('$O/c4_${v}_$i.json').read().strip().splitlines()[-1])['ms_per_step'])") $(grep 'sparse phases' $O/c4_${v}_$i.err | tail -1)"
  done
done
