#!/bin/bash
# Round 5: per-pivot end times of the FW beside the H2D (C3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05t}; mkdir -p $O
SRG_DEBUG_OVERLAP=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-ri --no-verify > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
grep -E "fw-overlap: (chunk 23|last)" $O/c3.err | tail -2
