#!/bin/bash
# Round-2 pass d: full GPU suite + smoke on HEAD, C1-C5 bench lines (C3 = default host entry with
# CPU baselines), rocprofv3 kernel stats of the default bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r02f}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 \
    > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt | cut -c1-200
timeout -k 10 300 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err || { tail -20 $out/bench_c3.err; exit 1; }
for c in c1 c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 > $out/bench_$c.json 2> $out/bench_$c.err || { tail -20 $out/bench_$c.err; exit 1; }
done
timeout -k 10 200 python -u bench.py --entry device --no-cpu --steps 10 > $out/bench_c3_device.json 2> $out/bench_c3_device.err || exit 1
for f in $out/bench_*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f', d.get('ms_per_step'), d.get('value'), (d.get('roofline') or {}).get('frac'))"; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 5 > "$GRAFT_REPO_ROOT/$out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$out/prof.err" \
    || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/$out/prof.err"; exit 1; }
echo all done
