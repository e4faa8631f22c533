#!/bin/bash
# A subset of the GPU suite (pytest -k / file args), log under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 "$@" \
    > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -25 $out/pytest_gpu.log
