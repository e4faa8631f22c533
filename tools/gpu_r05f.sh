#!/bin/bash
# Round 5: full pass with the host-entry key shipping, then a C3 A/B (u32 keys widened on the host
# vs u64 rows over PCIe)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05f}; mkdir -p $O
./tools/gpu_full.sh ${1:-r05f} || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu > $O/c3_keys_$i.json 2> $O/c3_keys_$i.err || exit 1
  SRG_NO_KEY_D2H=1 timeout -k 10 200 python -u bench.py --steps 10 --no-cpu > $O/c3_u64_$i.json 2> $O/c3_u64_$i.err || exit 1
done
cat $O/c3_*.json
