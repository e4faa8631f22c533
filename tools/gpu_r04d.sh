#!/bin/bash
# round 4 pass d: every new GPU test, then A/B numbers (overlap, fused step traces, sims, cold call)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04d}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 250 --timeout-method thread tests/test_fw_overlap.py tests/test_routing_info_keys.py tests/test_fw_step.py > $out/pytest_new.log 2>&1 || { echo "new tests failed"; tail -60 $out/pytest_new.log; exit 1; }
tail -4 $out/pytest_new.log
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 250 --timeout-method thread tests/test_sparse_gpu.py tests/test_gpu_parity.py -k "wide or large_latency or unit" > $out/pytest_wide.log 2>&1 || { echo "wide tests failed"; tail -60 $out/pytest_wide.log; exit 1; }
tail -4 $out/pytest_wide.log
for ov in 1 0; do
  SRG_DEBUG_OVERLAP=1 timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-verify --no-ri --fw-overlap $ov > $out/c3_ov$ov.json 2> $out/c3_ov$ov.err || { echo "c3 $ov failed"; tail -20 $out/c3_ov$ov.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c3_ov$ov.json')); b=d['breakdown_ms']; print('c3 ov$ov', d['ms_per_step'], 'h2d', b['ms_h2d'], 'build', b['ms_build'], 'fw', b['ms_fw'], 'scan', b['ms_scan'], 'frac', d['roofline']['frac'] if d['roofline'] else None, 'dev', d['device_entry_ms'])"
  grep "fw-overlap" $out/c3_ov$ov.err | tail -1
done
for sr in 8:0 4:0 2:0; do
  timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --simulate-rank $sr --fw-step 0 > $out/sim_${sr/:/_}_s0.json 2> $out/sim_${sr/:/_}_s0.err || { echo "sim $sr failed"; tail -20 $out/sim_${sr/:/_}_s0.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/sim_${sr/:/_}_s0.json')); b=d['breakdown_ms']; print('$sr step0', d['ms_per_step'], 'fw', b['ms_fw'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'xchg', b['ms_exchange'], 'd2h', b['ms_d2h'])"
done
bash tools/gpu_trace_step.sh ${1:-r04d}_trace
SRG_DEBUG_CREATE=1 SRG_DEBUG_CODEC=1 timeout -k 10 200 python3 -u tools/cold_probe2.py > $out/cold.json 2> $out/cold.err && cat $out/cold.json && grep -E "srg_create|codec" $out/cold.err | head -20
timeout -k 10 300 python3 -u bench.py --steps 3 --no-cpu --no-verify > $out/c3_ri.json 2> $out/c3_ri.err && python3 -c "import json; d=json.load(open('$out/c3_ri.json')); print('c3 host', d['ms_per_step'], 'ri', d['routing_info'])"
