#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-var}
mkdir -p $out
export SRG_DEBUG_CODEC=1
for i in 1 2; do
timeout -k 10 300 python -u bench.py > $out/b$i.json 2> $out/b$i.err || { tail -20 $out/b$i.err; exit 1; }
python -c "import json;d=json.load(open('$out/b$i.json'));print('default', d['ms_per_step'], d['breakdown_ms']['ms_h2d'])"; grep codec $out/b$i.err | tail -3
timeout -k 10 300 python -u bench.py --no-cpu > $out/n$i.json 2> $out/n$i.err || { tail -20 $out/n$i.err; exit 1; }
python -c "import json;d=json.load(open('$out/n$i.json'));print('no-cpu', d['ms_per_step'], d['breakdown_ms']['ms_h2d'])"; grep codec $out/n$i.err | tail -3
done
