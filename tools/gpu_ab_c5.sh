#!/bin/bash
# C5 A/B of the default library against ab/$1 (SRG_LIB_PATH) after the events parity tests.  usage: tools/gpu_ab_c5.sh LIB TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_events.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then L=$GRAFT_REPO_ROOT/ab/$1; else L=; fi
    SRG_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config c5 --steps 20 --no-cpu > $O/c5_${v}_$i.json 2> $O/c5_${v}_$i.err || { tail -5 $O/c5_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['step_ms']['median'] if 'step_ms' in d else '')"
  done
done
