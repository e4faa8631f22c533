#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-tune2}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "codec" --timeout 250 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
export SRG_DEBUG_CODEC=1
run() { timeout -k 10 200 python -u bench.py --no-cpu --steps 8 "$@" > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$out/b.json'));b=d['breakdown_ms'];print(sys.argv[1:], d['ms_per_step'], 'h2d', b['ms_h2d'])" "$@"; grep codec $out/b.err | tail -2; }
for i in 1 2 3 4; do run; done
run --h2d-codec 0
