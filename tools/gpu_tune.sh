#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-tune}
mkdir -p $out
export SRG_DEBUG_CODEC=1
run() { timeout -k 10 200 python -u bench.py --no-cpu --steps 8 "$@" > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys,os;d=json.load(open('$out/b.json'));b=d['breakdown_ms'];print(os.environ.get('SRG_CODEC_THREADS','8'), sys.argv[1:], d['ms_per_step'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'd2h', b['ms_d2h'])" "$@"; grep codec $out/b.err | tail -1; }
for t in 8 12 6 8 12; do SRG_CODEC_THREADS=$t run; done
run --scan-groups 4
run --scan-groups 2
