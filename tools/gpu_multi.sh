#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-multi}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_multi_gpu.py tests/test_sparse_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
