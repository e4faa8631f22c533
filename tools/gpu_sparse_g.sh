#!/bin/bash
# Sparse A/B of the two-phase kernel on C4 (device entry): bucket width divisors, with the per-phase
# wall-clock split the kernel reports under SRG_DEBUG_SPARSE.  usage: tools/gpu_sparse_g.sh TAG [div ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}; shift
O=gpurun_out/$TAG; mkdir -p $O
for d in "${@:-1}"; do
  SRG_DEBUG_SPARSE=1 timeout -k 10 300 python -u bench.py --config c4 --entry device --steps 3 --no-cpu --no-ri --sparse-delta-div $d > $O/c4_div$d.json 2> $O/c4_div$d.err || { tail -5 $O/c4_div$d.err; exit 1; }
  echo "div=$d $(python3 -c "import json; print(json.loads(open('$O/c4_div$d.json').read().strip().splitlines()[-1])['ms_per_step'])")"
  grep "sparse" $O/c4_div$d.err | tail -2
done
