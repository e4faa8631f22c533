#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-loss}
mkdir -p $out
run() { timeout -k 10 200 python -u bench.py --no-cpu --steps 4 "$@" > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$out/b.json'));print(sys.argv[1:], d['ms_per_step'], d['breakdown_ms'])" "$@"; }
run --entry device --loss-chunks 1
run --entry device --loss-chunks 8
run --entry host --loss-chunks 1
run --entry host --loss-chunks 8
run --entry host --loss-chunks 8 --d2h-mode 0
run --entry host --loss-chunks 32
