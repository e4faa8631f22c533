#!/bin/bash
# round 4: H2D/FW overlap tests + C3 A/B, then the fused-step traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04c}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 250 --timeout-method thread tests/test_fw_overlap.py > $out/pytest_ov.log 2>&1 || { echo "overlap tests failed"; tail -60 $out/pytest_ov.log; exit 1; }
tail -4 $out/pytest_ov.log
for ov in 1 0 1 0; do
  SRG_DEBUG_OVERLAP=1 timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-verify --fw-overlap $ov > $out/c3_ov$ov.json 2> $out/c3_ov$ov.err || { echo "c3 $ov failed"; tail -20 $out/c3_ov$ov.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c3_ov$ov.json')); b=d['breakdown_ms']; print('c3 ov$ov', d['ms_per_step'], 'h2d', b['ms_h2d'], 'build', b['ms_build'], 'fw', b['ms_fw'], 'scan', b['ms_scan'], 'frac', d['roofline']['frac'] if d['roofline'] else None)"
  grep "fw-overlap" $out/c3_ov$ov.err | tail -1
done
bash tools/gpu_trace_step.sh ${1:-r04c}_trace
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 250 --timeout-method thread tests/test_routing_info_keys.py > $out/pytest_ri.log 2>&1 || { echo "ri tests failed"; tail -60 $out/pytest_ri.log; exit 1; }
tail -4 $out/pytest_ri.log
SRG_DEBUG_CREATE=1 SRG_DEBUG_CODEC=1 timeout -k 10 200 python3 -u tools/cold_probe2.py > $out/cold.json 2> $out/cold.err && cat $out/cold.json && grep -E "srg_create|codec" $out/cold.err | head -20
