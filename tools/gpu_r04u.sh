#!/bin/bash
# round 4 pass u: bulk-tile k loop variant (interleaved pair adds, unroll 2): FW parity, C3 device/host
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04u}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fw or c3 or c2 or atlas" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri --entry device > $out/dev_$i.json 2> $out/dev_$i.err && python3 -c "import json; d=json.load(open('$out/dev_$i.json')); b=d['breakdown_ms']; r=d['roofline']; print('device', d['ms_per_step'], 'fw', b['ms_fw'], 'bulk', r['avg_launch_ms'], 'frac', r['frac'])"
timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri --no-verify > $out/host_$i.json 2> $out/host_$i.err && python3 -c "import json; d=json.load(open('$out/host_$i.json')); r=d['roofline']; print('host', d['ms_per_step'], 'bulk', r['avg_launch_ms'], 'frac', r['frac'])"
done
