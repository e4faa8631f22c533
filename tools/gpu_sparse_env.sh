#!/bin/bash
# Sparse parity tests on the default, then C4 device-entry lines alternating an environment
# variable's values (REPS rounds), with the per-phase split.  usage: tools/gpu_sparse_env.sh TAG VAR v1 v2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}; VAR=${2:?var}; shift 2
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    timeout -k 10 300 env $VAR=$v SRG_DEBUG_SPARSE=1 python -u bench.py --config c4 --entry device --steps 3 --no-cpu --no-ri > $O/c4_${v}_$i.json 2> $O/c4_${v}_$i.err || { tail -5 $O/c4_${v}_$i.err; exit 1; }
    echo "$VAR=$v $(python3 -c "import json; print(json.loads(open('$O/c4_${v}_$i.json').read().strip().splitlines()[-1])['ms_per_step'])")"
    grep "sparse phases" $O/c4_${v}_$i.err | tail -1
  done
done
