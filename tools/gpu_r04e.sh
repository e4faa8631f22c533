#!/bin/bash
# round 4 pass e: device-side exchange in the two-stream chain (tests + sims), C3 overlap timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04e}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 250 --timeout-method thread tests/test_fw_step.py tests/test_fw_overlap.py > $out/pytest.log 2>&1 || { echo "tests failed"; tail -60 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
for sr in 8:0 4:0 2:0; do
  for st in -1 0; do
    timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr --fw-step $st > $out/sim_${sr/:/_}_s$st.json 2> $out/sim_${sr/:/_}_s$st.err || { echo "sim $sr $st failed"; tail -20 $out/sim_${sr/:/_}_s$st.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/sim_${sr/:/_}_s$st.json')); b=d['breakdown_ms']; print('$sr step$st', d['ms_per_step'], 'fw', b['ms_fw'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'xchg', b['ms_exchange'], 'd2h', b['ms_d2h'], 'total', b['ms_total'])"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$out/tl -o c3ov -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu --no-verify --no-ri --fw-overlap 1 > $GRAFT_REPO_ROOT/$out/tl.log 2>&1 || { echo "timeline failed"; tail -20 $GRAFT_REPO_ROOT/$out/tl.log; exit 1; }
cd $GRAFT_REPO_ROOT
find $out/tl -name "*.csv" | head
