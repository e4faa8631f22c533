#!/bin/bash
# Cold call (srg_create + the first call on never-touched tables) with srg_create's warm-up on / off,
# alternating, REPS rounds (C3 host entry).  usage: tools/gpu_cold.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}; O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 ${REPS:-3}); do
  for w in 1 0; do
    timeout -k 10 200 env SRG_CREATE_WARM=$w SRG_DEBUG_CREATE=1 python -u bench.py --steps 3 --no-cpu --no-ri --no-verify > $O/warm${w}_$i.json 2> $O/warm${w}_$i.err || { tail -10 $O/warm${w}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/warm${w}_$i.json').read().strip().splitlines()[-1]); c=d['config']; print('warm$w', 'cold', c.get('cold_call_ms'), c.get('cold_call_breakdown_ms'), 'step', d['ms_per_step'], d['step_ms']['median'])"
  done
done
