#!/bin/bash
# Round 5: simulated rank 8:0 -- timing lines and a kernel trace of the FW chain (per-pivot breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05y}; mkdir -p $O
for s in 8:0 8:7; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --simulate-rank $s > $O/sim_${s/:/_}.json 2> $O/sim_${s/:/_}.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/sim_${s/:/_}.json').read().strip().splitlines()[-1]); print('$s', d['ms_per_step'], d['breakdown_ms'])"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -o sim8 -- python3 -u $GRAFT_REPO_ROOT/bench.py --steps 3 --no-cpu --no-ri --no-verify --simulate-rank 8:0 > $GRAFT_REPO_ROOT/$O/sim8_prof.json 2> $GRAFT_REPO_ROOT/$O/sim8_prof.err) || exit 1
python3 tools/kstats.py $O/stats/sim8_kernel_stats.csv fw_ k_hop k_line k_model tight_v5 k_loss_rows
