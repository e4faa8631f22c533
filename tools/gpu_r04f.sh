#!/bin/bash
# round 4 pass f: grouped catch-up (FW beside the H2D): tests, C3 A/B alternating, codec threads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04f}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 250 --timeout-method thread tests/test_fw_overlap.py > $out/pytest.log 2>&1 || { echo "tests failed"; tail -60 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for i in 1 2; do
for cfg in "ov1:--fw-overlap 1" "ov0:--fw-overlap 0" "ov1t16:--fw-overlap 1"; do
  name=${cfg%%:*}; args=${cfg#*:}
  if [ "$name" = "ov1t16" ]; then export SRG_CODEC_THREADS=16; else unset SRG_CODEC_THREADS; fi
  timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-verify --no-ri $args > $out/c3_${name}_$i.json 2> $out/c3_${name}_$i.err || { echo "c3 $name failed"; tail -20 $out/c3_${name}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c3_${name}_$i.json')); b=d['breakdown_ms']; print('$name', d['ms_per_step'], 'h2d', b['ms_h2d'], 'fw', b['ms_fw'], 'scan', b['ms_scan'], 'total', b['ms_total'], 'dev', d['device_entry_ms'])"
done
done
unset SRG_CODEC_THREADS
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o c3ov -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --fw-overlap 1 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
find $out/prof -name "*stats.csv" | head
