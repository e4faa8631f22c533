#!/bin/bash
# Round 5: sparse hub bounds (SRG_OPT_SPARSE_HUBS) -- parity tests, then C4 with 0 / 128 / 256 / 512 hubs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sparse_hubs.py tests/test_sparse_gpu.py -m gpu -x -v --timeout 250 --timeout-method thread > $O/pytest_hubs.log 2>&1 || { tail -40 $O/pytest_hubs.log; exit 1; }
tail -1 $O/pytest_hubs.log
export SRG_DEBUG_SPARSE=1
for h in 0 128 256 512; do
  timeout -k 10 400 python3 -u bench.py --config c4 --no-cpu --sparse-hubs $h > $O/c4_h$h.json 2> $O/c4_h$h.err || { tail -10 $O/c4_h$h.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_h$h.json').read().strip().splitlines()[-1]); print('hubs $h', d['ms_per_step'], d.get('breakdown_ms'), d.get('verified_rows'))"
  grep "sparse:" $O/c4_h$h.err | tail -1
done
