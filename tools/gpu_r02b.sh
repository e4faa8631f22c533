#!/bin/bash
# Round-2 pass b: full GPU suite (incl. C3 multi-rank G=2/8), C3-size GML ingest, full C1/C2 CPU baselines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r02b}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 \
    > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -18 $out/pytest_gpu.log
timeout -k 10 400 python -u tools/ingest/ingest_bench.py --vertices 10000 --dir /tmp > $out/ingest_c3.json 2> $out/ingest.err \
    && cat $out/ingest_c3.json || { tail -20 $out/ingest.err; exit 1; }
timeout -k 10 600 python -u tools/cpu_full.py > $out/cpu_full.json 2> $out/cpu_full.err && cat $out/cpu_full.json
