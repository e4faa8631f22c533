#!/bin/bash
# simulated-rank bench lines (modelled collectives): tools/gpu_sims.sh TAG "G:r ..." [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; sims=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for sr in $sims; do
    timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --simulate-rank $sr "$@" > $out/sim_${sr/:/_}.json 2> $out/sim_${sr/:/_}.err || { echo "sim $sr failed"; tail -20 $out/sim_${sr/:/_}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$out/sim_${sr/:/_}.json')); b=d['breakdown_ms']; print('$sr', d['ms_per_step'], 'fw', b['ms_fw'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'xchg', b['ms_exchange'], 'd2h', b['ms_d2h'])"
done
