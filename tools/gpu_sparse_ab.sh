#!/bin/bash
# Sparse A/B of two library builds on C4 (device entry): the tree's library against ab/libbase.so
# (SRG_LIB_PATH), alternating, after the sparse parity tests on the tree's.  usage: tools/gpu_sparse_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in $(seq 1 ${REPS:-2}); do
  for v in "new|" "base|SRG_LIB_PATH=ab/libbase.so"; do
    IFS='|' read -r name envs <<< "$v"
    timeout -k 10 300 env SRG_DEBUG_SPARSE=1 $envs python -u bench.py --config c4 --entry device --steps 3 --no-cpu --no-ri > $O/c4_${name}_$i.json 2> $O/c4_${name}_$i.err || { tail -5 $O/c4_${name}_$i.err; exit 1; }
    echo "$name $(python3 -c "import json; print(json.loads(open('$O/c4_${name}_$i.json').read().strip().splitlines()[-1])['ms_per_step'])")"
    grep "sparse phases" $O/c4_${name}_$i.err | tail -1
  done
done
