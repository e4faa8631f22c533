#!/bin/bash
# round 4 pass h: kernel time by kernel, C3 host entry with and without the FW beside the H2D
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04h}
mkdir -p $out
cd /tmp
for ov in 1 0; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ov$ov -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu --no-verify --no-ri --fw-overlap $ov > $out/ov$ov.log 2>&1 || { echo "prof $ov failed"; tail -20 $out/ov$ov.log; exit 1; }
done
find $out -name "*kernel_stats.csv"
