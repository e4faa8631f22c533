#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-v7b}
mkdir -p $out
run() { timeout -k 10 200 python -u bench.py --no-cpu --entry device --steps 5 "$@" > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$out/b.json'));print(sys.argv[1:], d['ms_per_step'], d['breakdown_ms']['ms_scan'])" "$@"; }
run --scan-variant 7
run --scan-variant 91
run --scan-variant 92
