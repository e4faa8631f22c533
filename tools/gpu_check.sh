#!/bin/bash
# One GPU-box pass: parity tests, smoke, the default bench line and a rocprofv3 kernel summary.
# Usage (from the repo root): gpurun --timeout 1100 -- 'bash tools/gpu_check.sh <tag>'
set -o pipefail
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$out/pytest_gpu.log"; exit 1; }
tail -3 "$out/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "$out/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 240 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" \
    || { echo "bench failed"; tail -30 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu > "$GRAFT_REPO_ROOT/$out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$out/prof.err" \
    || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/$out/prof.err"; exit 1; }
echo done
