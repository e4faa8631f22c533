#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/late3
mkdir -p $out
nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"
for cfg in "1 8" "1 16" "1 12" "0 8" "0 16" "1 8" "1 16" "1 12" "0 8" "0 16"; do
set -- $cfg
SRG_CODEC_THREADS=$2 timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 10 --late-loss $1 > $out/c3.json 2>$out/c3.err || { tail -20 $out/c3.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3.json'));b=d['breakdown_ms'];print('late $1 thr $2', d['ms_per_step'], 'h2d',b['ms_h2d'],'build',b['ms_build'],'fw',b['ms_fw'],'scan',b['ms_scan'])"
done
