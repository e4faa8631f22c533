#!/bin/bash
# round 4 pass w: same-box A/B of three k-loop builds (A2 = interleave 2, unroll 2;
# B = interleave 4, unroll 2; D = interleave 4, no unroll): C3 device and host entry, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04w}
mkdir -p $out
for i in 1 2; do
for v in A2 B D; do
  SRG_LIB_PATH=$GRAFT_REPO_ROOT/ab/lib$v.so timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri --no-verify --entry device > $out/dev_${v}_$i.json 2> $out/dev_${v}_$i.err || { echo "dev $v failed"; tail -5 $out/dev_${v}_$i.err; exit 1; }
  SRG_LIB_PATH=$GRAFT_REPO_ROOT/ab/lib$v.so timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri --no-verify > $out/host_${v}_$i.json 2> $out/host_${v}_$i.err || { echo "host $v failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/dev_${v}_$i.json')); h=json.load(open('$out/host_${v}_$i.json')); print('$v', 'device', d['ms_per_step'], 'fw', d['breakdown_ms']['ms_fw'], 'bulk', d['roofline']['avg_launch_ms'], '| host', h['ms_per_step'], 'bulk', h['roofline']['avg_launch_ms'])"
done
done
