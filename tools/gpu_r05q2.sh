#!/bin/bash
# Round 5: multi-rank bulk as 64 x 64 quadrants (SRG_BULK_Q=1) -- multi-rank parity with it on, then
# simulated ranks 8:0 / 4:0 with and without
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05q2}; mkdir -p $O
SRG_BULK_Q=1 timeout -k 10 900 python -u -m pytest tests/test_multi_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_multi.log 2>&1 || { tail -30 $O/pytest_multi.log; exit 1; }
tail -1 $O/pytest_multi.log
for s in 8:0 4:0 8:0; do
  for v in 0 1; do
    if [ $v = 1 ]; then export SRG_BULK_Q=1; else unset SRG_BULK_Q; fi
    timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --simulate-rank $s > $O/sim_${s/:/_}_q$v.json 2> $O/sim_${s/:/_}_q$v.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/sim_${s/:/_}_q$v.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$s q=$v', d['ms_per_step'], 'fw', b['ms_fw'], 'frac', d['roofline']['frac'], 'launch_ms', d['roofline']['avg_launch_ms'])"
  done
done
