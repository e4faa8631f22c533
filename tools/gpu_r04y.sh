#!/bin/bash
# round 4 closing pass on the interleaved k loop: rocprofv3 stats of the default C3 bench command,
# FW PMC passes (overlap off, full bulk launches), device entry, simulated ranks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04y}
mkdir -p $out
step() { echo "[$(date +%T)] $*"; }
step stats
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o c3 -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu > $out/bench_c3_under_rocprof.json 2> $out/stats.err) || { echo "stats failed"; tail -20 $out/stats.err; exit 1; }
step pmc_fw
timeout -k 10 900 bash tools/pmc_fw.sh $out/pmc_fw --fw-overlap 0 > $out/pmc_fw.log 2>&1 || { echo "pmc_fw failed"; tail -20 $out/pmc_fw.log; exit 1; }
step device
timeout -k 10 400 python3 -u bench.py --entry device --no-cpu --no-ri > $out/bench_c3_device.json 2> $out/bench_c3_device.err || { echo "device failed"; exit 1; }
step sims
for sr in 2:0 4:0 8:0 8:7; do
  timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr > $out/sim_${sr/:/_}.json 2> $out/sim_${sr/:/_}.err || { echo "sim $sr failed"; tail -10 $out/sim_${sr/:/_}.err; exit 1; }
done
step done
for f in $out/*.json; do python3 -c "import json,os; d=json.load(open('$f')); r=d.get('roofline') or {}; print(os.path.basename('$f'), d['ms_per_step'], 'frac', r.get('frac'), 'avg_launch_ms', r.get('avg_launch_ms'), {k: round(v, 2) for k, v in (d.get('breakdown_ms') or {}).items()})"; done
