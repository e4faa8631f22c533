#!/bin/bash
# round 4 pass n: pair relaxation as two 32-bit adds + v_min3: full GPU suite, C3 host/device, sims
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04n}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri > $out/c3_$i.json 2> $out/c3_$i.err || { echo "c3 failed"; tail -10 $out/c3_$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/c3_$i.json')); b=d['breakdown_ms']; r=d['roofline']; print('c3 host', d['ms_per_step'], 'dev', d['device_entry_ms'], 'bulk', r['avg_launch_ms'], 'frac', r['frac'], 'cold', d['config'].get('cold_call_ms'), d['config'].get('cold_call_breakdown_ms'))"
done
timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri --entry device > $out/c3_dev.json 2> $out/c3_dev.err && python3 -c "import json; d=json.load(open('$out/c3_dev.json')); b=d['breakdown_ms']; r=d['roofline']; print('c3 device', d['ms_per_step'], 'fw', b['ms_fw'], 'bulk', r['avg_launch_ms'], 'frac', r['frac'])"
for sr in 8:0 2:0; do
  timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr > $out/sim_${sr/:/_}.json 2> $out/sim_${sr/:/_}.err && python3 -c "import json; d=json.load(open('$out/sim_${sr/:/_}.json')); b=d['breakdown_ms']; print('$sr', d['ms_per_step'], 'fw', b['ms_fw'])"
done
SRG_LATENCY_UNIT=1 timeout -k 10 300 python3 -u bench.py --lat-scale 1000 --no-cpu --no-ri --steps 3 --entry device > $out/c3_u64.json 2> $out/c3_u64.err && python3 -c "import json; d=json.load(open('$out/c3_u64.json')); print('u64 device', d['ms_per_step'])"
