#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/v11
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "scan_variants or v5_equals" > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for v in 5 11 5 11; do
timeout -k 10 200 python -u bench.py --no-cpu --entry device --steps 10 --scan-variant $v > $out/c3_dev_v$v.json 2>$out/c3.err || { tail -20 $out/c3.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3_dev_v$v.json'));b=d['breakdown_ms'];print('dev v$v', d['ms_per_step'], 'fw',b['ms_fw'],'scan',b['ms_scan'],'loss',b['ms_loss'])"
done
for v in 5 11; do
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 10 --scan-variant $v > $out/c3_host_v$v.json 2>$out/c3.err || { tail -20 $out/c3.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3_host_v$v.json'));b=d['breakdown_ms'];print('host v$v', d['ms_per_step'], 'h2d',b['ms_h2d'],'fw',b['ms_fw'],'scan',b['ms_scan'],'d2h',b['ms_d2h'])"
done
