#!/bin/bash
# Round-2 GPU pass: full GPU suite (incl. full-size C3/C4/C5 parity), host- and device-entry C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r02}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=15 \
    > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -22 $out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --entry host --steps 5 --warmup 1 --no-cpu > $out/host.json 2> $out/host.err && cat $out/host.json && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $out/dev.json 2> $out/dev.err && cat $out/dev.json
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 3 > "$GRAFT_REPO_ROOT/$out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$out/prof.err" \
    || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/$out/prof.err"; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-60,300-
