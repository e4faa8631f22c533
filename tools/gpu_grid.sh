#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-grid}
mkdir -p $out
run() { timeout -k 10 200 python -u bench.py --no-cpu --config c4 --steps 2 > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,os;d=json.load(open('$out/b.json'));r=d['roofline'];print(os.environ.get('SRG_SPARSE_GRID','default'), d['ms_per_step'], 'kernel', r['avg_launch_ms'])"; }
run
SRG_SPARSE_GRID=0 run
SRG_SPARSE_GRID=448 run
SRG_SPARSE_GRID=782 run
SRG_SPARSE_GRID=300 run
