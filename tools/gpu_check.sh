#!/bin/bash
# GPU suite + the C3 headline bench line, logs under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-check}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 \
    > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -20 $out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu > $out/c3.json 2> $out/c3.err && cat $out/c3.json
