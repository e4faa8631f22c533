#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-c4}
mkdir -p $out
shift
timeout -k 10 300 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
run() { timeout -k 10 200 python -u bench.py --no-cpu --config c4 --steps 2 "$@" > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$out/b.json'));r=d['roofline'];print(sys.argv[1:], d['ms_per_step'], 'kernel', r['avg_launch_ms'], 'frac', r['frac'], d.get('loss_rounds'))" "$@"; }
run --sparse-wgs 2 --sparse-group 8
run --sparse-wgs 1 --sparse-group 8
run --sparse-wgs 1 --sparse-group 4
run --sparse-wgs 2 --sparse-group 4
