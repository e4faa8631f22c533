#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-codec2}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "codec" --timeout 250 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
run() { timeout -k 10 200 python -u bench.py --no-cpu --steps 5 "$@" > $out/b.json 2>$out/b.err || { tail -20 $out/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$out/b.json'));print(sys.argv[1:], d['ms_per_step'], 'h2d', d['breakdown_ms']['ms_h2d'])" "$@"; grep codec $out/b.err | tail -2; }
export SRG_DEBUG_CODEC=1
for t in 8 4 16 8; do SRG_CODEC_THREADS=$t run --h2d-codec 1; done
run --h2d-codec 0
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
