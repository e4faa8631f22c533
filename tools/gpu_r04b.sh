#!/bin/bash
# round 4: fused FW step -- sims and C3/C2 A/B (step 1 = fused, 0 = two-stream), then the parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04b}
mkdir -p $out
for st in 1 0; do
  for sr in 8:0 4:0 2:0; do
    timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --simulate-rank $sr --fw-step $st > $out/sim_${sr/:/_}_s$st.json 2> $out/sim_${sr/:/_}_s$st.err || { echo "sim $sr $st failed"; tail -20 $out/sim_${sr/:/_}_s$st.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/sim_${sr/:/_}_s$st.json')); b=d['breakdown_ms']; print('$sr step$st', d['ms_per_step'], 'fw', b['ms_fw'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'xchg', b['ms_exchange'], 'd2h', b['ms_d2h'])"
  done
done
for st in 1 0; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-verify --fw-step $st > $out/c3_s$st.json 2> $out/c3_s$st.err || { echo "c3 $st failed"; tail -20 $out/c3_s$st.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c3_s$st.json')); b=d['breakdown_ms']; print('c3 step$st', d['ms_per_step'], 'dev', d['device_entry_ms'], 'fw', b['ms_fw'], 'h2d', b['ms_h2d'], 'frac', d['roofline']['frac'])"
  timeout -k 10 200 python3 -u bench.py --config c2 --steps 5 --no-cpu --no-verify --fw-step $st > $out/c2_s$st.json 2> $out/c2_s$st.err || { echo "c2 $st failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c2_s$st.json')); b=d['breakdown_ms']; print('c2 step$st', d['ms_per_step'], 'dev', d['device_entry_ms'], 'fw', b['ms_fw'])"
  timeout -k 10 200 python3 -u bench.py --config c1 --steps 5 --no-cpu --no-verify --fw-step $st > $out/c1_s$st.json 2> $out/c1_s$st.err || { echo "c1 $st failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c1_s$st.json')); b=d['breakdown_ms']; print('c1 step$st', d['ms_per_step'], 'dev', d['device_entry_ms'], 'fw', b['ms_fw'])"
done
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_multi_gpu.py > $out/pytest_multi.log 2>&1 || { echo "multi tests failed"; tail -60 $out/pytest_multi.log; exit 1; }
tail -5 $out/pytest_multi.log
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 250 --timeout-method thread tests/test_fw_step.py > $out/pytest_fw_step.log 2>&1 || { echo "fw_step tests failed"; tail -60 $out/pytest_fw_step.log; exit 1; }
tail -5 $out/pytest_fw_step.log
