#!/bin/bash
# GPU suite only (parity), log under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-tests}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=10 \
    > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -14 $out/pytest_gpu.log
