#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-v7}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "scan_variants or golden" --timeout 200 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
run() { timeout -k 10 200 python -u bench.py --no-cpu --entry device --steps 5 "$@" > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$out/b.json'));print(sys.argv[1:], d['ms_per_step'], d['breakdown_ms']['ms_scan'])" "$@"; }
run --scan-variant 5
run --scan-variant 9
run --scan-variant 9
run --scan-variant 5
