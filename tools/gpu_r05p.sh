#!/bin/bash
# Round 5: FW-overlap timeline (chunk landing vs pivots) of C3 with the fused encoder
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05p}; mkdir -p $O
SRG_DEBUG_OVERLAP=1 SRG_DEBUG_CODEC=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-ri --no-verify > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
grep -E "fw-overlap|codec:" $O/c3.err | tail -32
