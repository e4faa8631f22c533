#!/bin/bash
# round 4 pass p: block-row splits on the H2D stream: overlap tests + C3 A/B against the overlap off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04p}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_events.py tests/test_fw_overlap.py tools/dbg/test_ov_after.py tests/test_fw_step.py > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2 3; do
for ov in 1 0; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-verify --no-ri --fw-overlap $ov > $out/c3_ov${ov}_$i.json 2> $out/c3_ov${ov}_$i.err || { echo "c3 $ov failed"; tail -20 $out/c3_ov${ov}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c3_ov${ov}_$i.json')); b=d['breakdown_ms']; print('ov$ov', d['ms_per_step'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'total', b['ms_total'])"
done
done
SRG_DEBUG_OVERLAP=1 timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu --no-verify --no-ri --fw-overlap 1 > $out/c3dbg.json 2> $out/c3dbg.err && grep "last pivot" $out/c3dbg.err | tail -2
