#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-relabel}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
run() { timeout -k 10 200 python -u bench.py --no-cpu --config c4 --steps 2 "$@" > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$out/b.json'));r=d['roofline'];print(sys.argv[1:], d['ms_per_step'], 'kernel', r['avg_launch_ms'], 'frac', r['frac'], 'build', d['breakdown_ms']['ms_build'])" "$@"; }
run --sparse-relabel 1
run --sparse-relabel 0
run --sparse-relabel 1 --sparse-delta-div 2
run --sparse-relabel 1 --sparse-group 4
