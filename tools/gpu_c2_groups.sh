#!/bin/bash
# C2 host entry: scan-group counts alternated on one box (round 6)
cd $GRAFT_REPO_ROOT; O=gpurun_out/c2g; mkdir -p $O
for i in 1 2; do for g in 3 2 1 4; do
timeout -k 10 200 python -u bench.py --config c2 --steps 10 --no-cpu --no-ri --scan-groups $g > $O/c2_${g}_$i.json 2> $O/c2_${g}_$i.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c2_${g}_$i.json').read().strip().splitlines()[-1]); print('groups $g', d['ms_per_step'], d['step_ms']['median'], d['breakdown_ms']['ms_scan'], d['breakdown_ms']['ms_d2h'], d.get('verified_rows',{}).get('bit_exact'))"
done; done
