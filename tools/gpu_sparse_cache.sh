#!/bin/bash
# sparse cache-policy A/B (round 6): parity tests, then C4 lines for env settings and an alternative build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-scache}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, env...
  n=$1; shift
  env "$@" SRG_DEBUG_SPARSE=1 timeout -k 10 300 python -u bench.py --config c4 --entry device --steps 3 --no-cpu --no-ri > $O/c4_$n.json 2> $O/c4_$n.err || { tail -5 $O/c4_$n.err; exit 1; }
  echo "$n $(python3 -c "import json; print(json.loads(open('$O/c4_$n.json').read().strip().splitlines()[-1])['ms_per_step'])") $(grep 'sparse phases' $O/c4_$n.err | tail -1)"
}
for i in 1 2; do
  run base_$i X=0
  run wpc1_$i SRG_DS_WPC=1
  run ntinit_$i SRG_DS_NTINIT=1
  run bf_$i SRG_SPARSE_KERNEL=bf
  run bfnt_$i SRG_SPARSE_KERNEL=bf SRG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libbfnt.so
done
