#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-sim8b}
mkdir -p $out
for r in 0 7; do
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 3 --simulate-rank 8:$r > $out/h$r.json 2>$out/h$r.err || { tail -20 $out/h$r.err; exit 1; }
python -c "import json;d=json.load(open('$out/h$r.json'));print('host 8:$r', d['ms_per_step'], d['breakdown_ms'])"
timeout -k 10 200 python -u bench.py --no-cpu --entry device --steps 3 --simulate-rank 8:$r > $out/d$r.json 2>$out/d$r.err || { tail -20 $out/d$r.err; exit 1; }
python -c "import json;d=json.load(open('$out/d$r.json'));print('device 8:$r', d['ms_per_step'], d['breakdown_ms'])"
done
for r in 0 1; do
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 3 --simulate-rank 2:$r > $out/h2_$r.json 2>$out/h2_$r.err || { tail -20 $out/h2_$r.err; exit 1; }
python -c "import json;d=json.load(open('$out/h2_$r.json'));print('host 2:$r', d['ms_per_step'], d['breakdown_ms'])"
done
