#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/cuts2
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "host_entry or late_loss or h2d_codec" > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for cuts in "" "24,56" "" "24,56" "" "24,56"; do
SRG_SCAN_CUTS=$cuts timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 10 > $out/c3.json 2>$out/c3.err || { tail -20 $out/c3.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3.json'));b=d['breakdown_ms'];print('cuts [$cuts]', d['ms_per_step'], 'h2d',b['ms_h2d'],'fw',b['ms_fw'],'scan',b['ms_scan'],'d2h',b['ms_d2h'])"
done
timeout -k 10 200 python -u bench.py --no-cpu --config c2 --steps 10 > $out/c2.json 2>$out/c2.err || { tail -20 $out/c2.err; exit 1; }
python -c "import json;d=json.load(open('$out/c2.json'));b=d['breakdown_ms'];print('c2', d['ms_per_step'], b)"
