#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/late2
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "late_loss" > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for cfg in "1 64" "1 256" "0 0" "1 1024" "1 64" "1 256" "0 0" "1 1024"; do
set -- $cfg
SRG_WL_GRID=$2 timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 10 --late-loss $1 > $out/c3.json 2>$out/c3.err || { tail -20 $out/c3.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3.json'));b=d['breakdown_ms'];print('late $1 grid $2', d['ms_per_step'], 'h2d',b['ms_h2d'],'build',b['ms_build'],'fw',b['ms_fw'],'scan',b['ms_scan'])"
done
