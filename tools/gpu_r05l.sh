#!/bin/bash
# Round 5: simulated-rank test + the simulated-rank bench lines (the final pass stopped at sim 2:0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r05final}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_fw_xcd_order.py -x -v --timeout 120 --timeout-method thread > $out/pytest_sim.log 2>&1 || { tail -30 $out/pytest_sim.log; exit 1; }
tail -2 $out/pytest_sim.log
for sr in 2:0 2:1 4:0 4:3 8:0 8:7; do
  timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr > $out/sim_${sr/:/_}.json 2> $out/sim_${sr/:/_}.err || { echo "sim $sr failed"; tail -10 $out/sim_${sr/:/_}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/sim_${sr/:/_}.json')); b=d['breakdown_ms']; print('$sr', d['ms_per_step'], 'fw', b['ms_fw'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'xchg', b['ms_exchange'], 'd2h', b['ms_d2h'])"
done
