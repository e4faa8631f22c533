#!/bin/bash
# round 4 pass t: early closure (pivot tile first): rank tests, sims A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04t}
mkdir -p $out
GPU_MAX_HW_QUEUES=16 timeout -k 10 240 python3 -u tests/fw_step_ranks.py > $out/ranks.json 2> $out/ranks.err || { echo "ranks failed"; tail -20 $out/ranks.err; exit 1; }
python3 -c "
import json
r=json.load(open('$out/ranks.json')); print('rank cases ok:', sum(x['ok'] for x in r), 'of', len(r)); [print('BAD', x['case'], x['errors']) for x in r if not x['ok']]"
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 250 --timeout-method thread tests/test_multi_gpu.py > $out/pytest_multi.log 2>&1 || { echo "multi tests failed"; tail -30 $out/pytest_multi.log; exit 1; }
tail -1 $out/pytest_multi.log
for sr in 8:0 4:0 2:0 8:7; do
for ec in 1 0; do
  SRG_EARLY_CLOSE=$ec timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr > $out/sim_${sr/:/_}_e$ec.json 2> $out/sim_${sr/:/_}_e$ec.err || { echo "sim $sr failed"; tail -10 $out/sim_${sr/:/_}_e$ec.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/sim_${sr/:/_}_e$ec.json')); b=d['breakdown_ms']; print('$sr early$ec', d['ms_per_step'], 'fw', b['ms_fw'], 'total', b['ms_total'])"
done
done
