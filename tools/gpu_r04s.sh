#!/bin/bash
# round 4 pass s: D2H over two SDMA engines vs one (host entry), early-rows tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04s}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_entry or d2h or late_loss or codec" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2 3; do
for e in 2 1; do
  SRG_SDMA_ENGINES=$e timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-verify --no-ri > $out/c3_e${e}_$i.json 2> $out/c3_e${e}_$i.err || { echo "c3 $e failed"; tail -20 $out/c3_e${e}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c3_e${e}_$i.json')); b=d['breakdown_ms']; print('engines$e', d['ms_per_step'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'd2h', b['ms_d2h'], 'total', b['ms_total'], 'dev', d['device_entry_ms'])"
done
done
