#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-u64}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
timeout -k 10 300 python -u bench.py --entry device --steps 3 --warmup 1 --no-cpu --lat-scale 1000 > $out/c3_u64.json 2> $out/c3_u64.err \
    && python -c "import json;d=json.load(open('$out/c3_u64.json'));print('u64', d['ms_per_step'], d['breakdown_ms'], d['roofline']['frac'])" || { tail -20 $out/c3_u64.err; exit 1; }
