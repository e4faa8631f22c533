#!/bin/bash
# C2 (atlas_like(4096)) host-entry A/B: quadrant bulk on / off x chain line split, alternating,
# REPS rounds.  usage: tools/gpu_c2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}; O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 ${REPS:-3}); do
  for v in "q1s4|SRG_FW_BULK_Q=1|" "q0s4|SRG_FW_BULK_Q=0|" "q1s2|SRG_FW_BULK_Q=1|--fw-line-split 2" "q0s2|SRG_FW_BULK_Q=0|--fw-line-split 2"; do
    IFS='|' read -r name envs flags <<< "$v"
    timeout -k 10 200 env $envs python -u bench.py --config c2 --steps 10 --no-cpu --no-ri $flags > $O/${name}_$i.json 2> $O/${name}_$i.err || { tail -10 $O/${name}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${name}_$i.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('$name', d['ms_per_step'], d['step_ms']['median'], 'dev', d['device_entry_ms'], 'fw', d['breakdown_ms']['ms_fw'], 'frac', r.get('frac'), 'launch', r.get('avg_launch_ms'), d['verified_rows']['bit_exact'])"
  done
done
