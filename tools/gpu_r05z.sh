#!/bin/bash
# Round 5: simulated rank 8:0 -- host enqueue time of the FW loop vs its run time (is the chain launch bound?)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05z}; mkdir -p $O
export SRG_DEBUG_ENQ=1
timeout -k 10 200 python -u bench.py --steps 5 --no-cpu --no-ri --simulate-rank 8:0 > $O/sim_enq.json 2> $O/sim_enq.err || exit 1
grep "fw enqueue" $O/sim_enq.err | tail -4
timeout -k 10 200 python -u bench.py --steps 3 --no-cpu --no-ri --entry device > $O/c3_enq.json 2> $O/c3_enq.err || exit 1
grep "fw enqueue" $O/c3_enq.err | tail -2
