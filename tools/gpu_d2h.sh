#!/bin/bash
# D2H copy-kernel sweep on the C3 host entry + its parity test + a kernel trace at the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-d2h}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "host_entry_early or c2_sampled or device_entry" --timeout 200 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for w in 1 0 1; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 5 --d2h-mode $w > $out/b$w.json 2>$out/b$w.err || { tail -20 $out/b$w.err; exit 1; }
  python -c "import json;d=json.load(open('$out/b$w.json'));print('wgs $w', d['ms_per_step'], d['breakdown_ms'])"
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 3 > "$GRAFT_REPO_ROOT/$out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$out/prof.err" \
    || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/$out/prof.err"; exit 1; }
