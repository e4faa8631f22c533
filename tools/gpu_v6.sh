set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/v6
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "scan_variants or golden or scan_v5 or fw_symmetric" --timeout 200 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for v in 5 6 2 6; do timeout -k 10 120 python -u bench.py --entry device --steps 5 --no-cpu --scan-variant $v > $out/b$v.json 2>$out/b$v.err && python -c "
import json;d=json.load(open('$out/b$v.json'));r=d['roofline'];print('scan v$v', d['ms_per_step'], d['breakdown_ms'])" || exit 1; done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --entry device --no-cpu --steps 3 --scan-variant 6 > "$GRAFT_REPO_ROOT/$out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$out/prof.err" \
    || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/$out/prof.err"; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/rocpd_stats.py $(find $out/prof -name "*.db" | head -1) x "" | head -14
