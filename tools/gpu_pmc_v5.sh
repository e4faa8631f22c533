# PMC + kernel trace of the C3 device step with scan variant 5
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/pmc_v5
mkdir -p $out
bash tools/pmc_scan.sh $out --entry device --scan-variant 5 && python tools/pmc_kernel.py $out tight_v5 > $out/tight_v5_pmc.txt && cat $out/tight_v5_pmc.txt
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --entry device --no-cpu --steps 3 --scan-variant 5 > "$GRAFT_REPO_ROOT/$out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$out/prof.err" \
    || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/$out/prof.err"; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); head -14 "$f" | cut -c1-70,200-330
