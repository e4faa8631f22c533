#!/bin/bash
# Sparse parity tests, then C4 device-entry lines with the hub bounds on / off (SRG_SPARSE_HUBS),
# alternating, with the per-phase split (SRG_DEBUG_SPARSE).  usage: tools/gpu_sparse_hubs.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in $(seq 1 ${REPS:-2}); do
  for h in 1 0; do
    SRG_SPARSE_HUBS=$h SRG_DEBUG_SPARSE=1 timeout -k 10 300 python -u bench.py --config c4 --entry device --steps 3 --no-cpu --no-ri > $O/c4_h${h}_$i.json 2> $O/c4_h${h}_$i.err || { tail -5 $O/c4_h${h}_$i.err; exit 1; }
    echo "hubs=$h $(python3 -c "import json; print(json.loads(open('$O/c4_h${h}_$i.json').read().strip().splitlines()[-1])['ms_per_step'])")"
    grep "sparse" $O/c4_h${h}_$i.err | tail -3
  done
done
