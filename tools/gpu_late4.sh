#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/late4
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_multi_gpu.py -k "late_loss or h2d_codec or host_entry or edge_shard" > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for ll in 1 0 1 0 1 0 1 0; do
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 10 --late-loss $ll > $out/c3_late$ll.json 2>$out/c3.err || { tail -20 $out/c3.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3_late$ll.json'));b=d['breakdown_ms'];print('late $ll', d['ms_per_step'], 'h2d',b['ms_h2d'],'build',b['ms_build'],'fw',b['ms_fw'],'scan',b['ms_scan'],'frac',d['roofline']['frac'])"
done
