#!/bin/bash
# round 4 pass g: FW beside the H2D progress curve (SRG_DEBUG_OVERLAP)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04g}
mkdir -p $out
SRG_DEBUG_OVERLAP=1 timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu --no-verify --no-ri --fw-overlap 1 > $out/c3.json 2> $out/c3.err || { echo "c3 failed"; tail -20 $out/c3.err; exit 1; }
grep "fw-overlap" $out/c3.err | tail -30
