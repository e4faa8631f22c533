#!/bin/bash
# Round-2 pass c: full GPU suite + smoke on HEAD, default bench (C3 host entry), rocprofv3 kernel stats
# of the same command, C4 device bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r02c}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 \
    > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -4 $out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
timeout -k 10 300 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err && cat $out/bench_c3.json || { tail -20 $out/bench_c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --no-cpu --steps 3 > $out/bench_c4.json 2> $out/bench_c4.err && cat $out/bench_c4.json || { tail -20 $out/bench_c4.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 5 > "$GRAFT_REPO_ROOT/$out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$out/prof.err" \
    || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/$out/prof.err"; exit 1; }
cd $GRAFT_REPO_ROOT
find $out/prof -name "*stats*" | head
