#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/shard2
mkdir -p $out
for cfg in 8:0 8:7 4:0 4:3; do
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 3 --simulate-rank $cfg > $out/h$cfg.json 2>$out/h$cfg.err || { tail -20 $out/h$cfg.err; exit 1; }
python -c "import json;d=json.load(open('$out/h$cfg.json'));print('host $cfg', d['ms_per_step'], d['breakdown_ms'])"
done
