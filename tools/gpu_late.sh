#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/late
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "late_loss or h2d_codec or host_entry" > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -3 $out/pytest.txt
for ll in 1 0 1 0; do
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 10 --late-loss $ll > $out/c3_late$ll.json 2>$out/c3_late$ll.err || { tail -20 $out/c3_late$ll.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3_late$ll.json'));print('late $ll', d['ms_per_step'], d['breakdown_ms'])"
done
