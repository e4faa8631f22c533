#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-sim8}
mkdir -p $out
for r in 0 7; do
timeout -k 10 200 python -u bench.py --no-cpu --entry device --steps 3 --simulate-rank 8:$r > $out/s$r.json 2>$out/s$r.err || { tail -20 $out/s$r.err; exit 1; }
cat $out/s$r.json
done
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 3 --simulate-rank 8:0 > $out/h0.json 2>$out/h0.err || { tail -20 $out/h0.err; exit 1; }
cat $out/h0.json
