#!/bin/bash
# Sparse-path A/B on the GPU box: the sparse parity tests on the default kernel, then C4 device-entry
# bench lines alternating the two-phase kernel (default) with the lexicographic sweeps
# (SRG_SPARSE_KERNEL=bf), with the kernels' own counters (SRG_DEBUG_SPARSE) in the .err files.
#   usage: tools/gpu_sparse.sh TAG [pytest-args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread "$@" > $O/pytest_sparse.log 2>&1 || { tail -40 $O/pytest_sparse.log; exit 1; }
tail -2 $O/pytest_sparse.log
for i in $(seq 1 ${REPS:-2}); do
  for v in "ds|" "bf|SRG_SPARSE_KERNEL=bf"; do
    IFS='|' read -r name envs <<< "$v"
    timeout -k 10 300 env SRG_DEBUG_SPARSE=1 $envs python -u bench.py --config c4 --entry device --steps 3 --no-cpu --no-ri ${BENCH_FLAGS} > $O/c4_${name}_$i.json 2> $O/c4_${name}_$i.err || { tail -20 $O/c4_${name}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c4_${name}_$i.json').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], d.get('verified_rows'))"
    grep -m1 "^sparse:" $O/c4_${name}_$i.err || true
  done
done
