#!/bin/bash
# Round-2 pass e: multi-rank + sparse GPU tests, the u64-key C3 bench, C3-size GML ingest, full C1/C2 CPU baselines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r02e}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_multi_gpu.py tests/test_sparse_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
timeout -k 10 300 python -u bench.py --entry device --steps 3 --warmup 1 --no-cpu --lat-scale 1000 > $out/c3_u64.json 2> $out/c3_u64.err \
    && python -c "import json;d=json.load(open('$out/c3_u64.json'));print('u64', d['ms_per_step'], d['config']['path'], d['roofline']['frac'])" || { tail -20 $out/c3_u64.err; exit 1; }
timeout -k 10 500 python -u tools/ingest/ingest_bench.py --vertices 10000 --dir /tmp > $out/ingest_c3.json 2> $out/ingest.err \
    && cat $out/ingest_c3.json || { tail -20 $out/ingest.err; exit 1; }
timeout -k 10 700 python -u tools/cpu_full.py > $out/cpu_full.json 2> $out/cpu_full.err && cat $out/cpu_full.json
