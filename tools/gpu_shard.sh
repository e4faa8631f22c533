#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/shard
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_multi_gpu.py > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -3 $out/pytest.txt
for r in 0 7; do
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 3 --simulate-rank 8:$r > $out/h$r.json 2>$out/h$r.err || { tail -20 $out/h$r.err; exit 1; }
python -c "import json;d=json.load(open('$out/h$r.json'));print('host 8:$r', d['ms_per_step'], d['breakdown_ms'])"
done
for r in 0 3; do
timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 3 --simulate-rank 4:$r > $out/h4_$r.json 2>$out/h4_$r.err || { tail -20 $out/h4_$r.err; exit 1; }
python -c "import json;d=json.load(open('$out/h4_$r.json'));print('host 4:$r', d['ms_per_step'], d['breakdown_ms'])"
done
